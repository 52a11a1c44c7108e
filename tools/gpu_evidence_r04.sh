# Round-4 evidence at the current tree (after tools/gpu_r04.sh passed): PMC traffic
# (FETCH_SIZE, WRITE_SIZE) and SQ occupancy / issue counters of the 1080p x 8 workload and of
# 4K x 2, the bench line reading the traffic, and rocprofv3 kernel statistics of a 1080p-only
# bench run (per configuration).  Every GPU step time-limited; any failure ends the script.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc gpurun_out/pmc4k gpurun_out/prof gpurun_out/pmcsq
export TMPDIR=/tmp
export AV1R_GIT_HEAD=${AV1R_GIT_HEAD:-unknown}
B1080="--steps 8 --warmup 2 --frames 12 --no-cpu --no-4k --ivf-frames 0 --output-steps 0"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc/$c -o run -- \
        python3 bench.py $B1080 > gpurun_out/pmc/$c.json 2> gpurun_out/pmc/$c.err || exit $?
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc4k/$c -o run -- \
        python3 bench.py --config 4k --streams 2 --frames 12 --steps 6 --warmup 2 --no-cpu --ivf-frames 0 --output-steps 0 > gpurun_out/pmc4k/$c.json 2> gpurun_out/pmc4k/$c.err || exit $?
done
python3 tools/pmc_traffic.py gpurun_out/pmc gpurun_out/traffic.json 8 1080p > /dev/null || exit $?
python3 tools/pmc_traffic.py gpurun_out/pmc4k gpurun_out/traffic_4k.json 2 4k > /dev/null || exit $?
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcsq/g$i -o run -- \
        python3 bench.py $B1080 > gpurun_out/pmcsq/g$i.json 2> gpurun_out/pmcsq/g$i.err || exit $?
done
python3 tools/pmc_sq_report.py gpurun_out/pmcsq > gpurun_out/pmcsq/report.txt || exit $?
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 --traffic gpurun_out/traffic.json --traffic-4k gpurun_out/traffic_4k.json > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 --traffic gpurun_out/traffic.json > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || exit $?
find gpurun_out/prof -name "*kernel_stats.csv"
cat gpurun_out/pmcsq/report.txt
