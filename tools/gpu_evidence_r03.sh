# Round-3 evidence: PMC traffic (FETCH_SIZE, WRITE_SIZE passes; kernel counters only) of the
# 1080p and 4K 4x2-tile workloads, the default bench line reading them, and a rocprofv3
# kernel-trace/stats run of the bench (the same command).  Every GPU step time-limited.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc gpurun_out/pmc4k gpurun_out/prof
export TMPDIR=/tmp
export AV1R_GIT_HEAD=${AV1R_GIT_HEAD:-02fed5c}
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc/$c -o run -- \
        python3 bench.py --steps 8 --warmup 2 --frames 12 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 > gpurun_out/pmc/$c.json 2> gpurun_out/pmc/$c.err || exit $?
    timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc4k/$c -o run -- \
        python3 bench.py --config 4k --streams 2 --frames 12 --steps 6 --warmup 2 --no-cpu --ivf-frames 0 --output-steps 0 > gpurun_out/pmc4k/$c.json 2> gpurun_out/pmc4k/$c.err || exit $?
done
python3 tools/pmc_traffic.py gpurun_out/pmc gpurun_out/traffic.json 8 1080p > /dev/null || exit $?
python3 tools/pmc_traffic.py gpurun_out/pmc4k gpurun_out/traffic_4k.json 2 4k > /dev/null || exit $?
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --traffic gpurun_out/traffic.json --traffic-4k gpurun_out/traffic_4k.json > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu --traffic gpurun_out/traffic.json --traffic-4k gpurun_out/traffic_4k.json > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || exit $?
find gpurun_out/prof -name "*kernel_stats.csv"
