# SQ counters per kernel (one pass per group, kernel counters only); folded by
# tools/pmc_sq_report.py
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcsq
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcsq/g$i -o run -- \
        python3 bench.py --steps 4 --warmup 1 --frames 4 --no-cpu --streams 8 > gpurun_out/pmcsq/g$i.json 2> gpurun_out/pmcsq/g$i.err
    rc=$?
    echo "group $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmcsq/g$i.err; exit $rc; fi
done
python3 tools/pmc_sq_report.py gpurun_out/pmcsq
