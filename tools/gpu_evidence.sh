# Round evidence in one call: PMC traffic passes (FETCH_SIZE, WRITE_SIZE; kernel counters
# only) folded per stage, the default bench line (with CPU baseline) reading that traffic,
# and a rocprofv3 kernel-trace/stats run of the bench.  Every GPU step time-limited.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc gpurun_out/prof
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc/$c -o run -- \
        python3 bench.py --steps 8 --warmup 2 --frames 12 --no-cpu > gpurun_out/pmc/$c.json 2> gpurun_out/pmc/$c.err || exit $?
done
python3 tools/pmc_traffic.py gpurun_out/pmc gpurun_out/traffic.json 8 > /dev/null || exit $?  # (AV1R_GIT_HEAD: set by the caller)
timeout -k 10 600 python3 bench.py --traffic gpurun_out/traffic.json > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --no-cpu --traffic gpurun_out/traffic.json > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || exit $?
find gpurun_out/prof -name "*kernel_stats.csv"
