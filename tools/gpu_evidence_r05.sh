# Round-5 SQ evidence: one rocprofv3 --pmc pass per counter group, each a bench run with the
# same fixed work (--prime-steps), every ratio computed within one pass (tools/pmc_sq_report.py).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcsq
export TMPDIR=/tmp
B1080="--steps 8 --warmup 2 --frames 60 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 --prime-steps 1"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcsq/g$i -o run -- \
        python3 bench.py $B1080 > gpurun_out/pmcsq/g$i.json 2> gpurun_out/pmcsq/g$i.err || exit $?
done
python3 tools/pmc_sq_report.py gpurun_out/pmcsq > gpurun_out/pmcsq/report.txt || exit $?
cat gpurun_out/pmcsq/report.txt
