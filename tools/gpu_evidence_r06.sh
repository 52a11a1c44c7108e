# Round-6 evidence at the current tree: the GPU suite, then PMC traffic (FETCH_SIZE, WRITE_SIZE)
# of the 1080p x 8 and 4K x 2 workloads, the SQ passes (fixed work per pass), the default bench
# line reading the traffic, and rocprofv3 kernel statistics of a 1080p-only bench.  Every GPU
# step time-limited; any failure ends the script.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc gpurun_out/pmc4k gpurun_out/prof gpurun_out/pmcsq
export TMPDIR=/tmp
export AV1R_GIT_HEAD=${AV1R_GIT_HEAD:-unknown}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { tail -40 gpurun_out/pytest.log; exit 1; }
tail -2 gpurun_out/pytest.log
B1080="--steps 8 --warmup 2 --frames 12 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 --prime-steps 1"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc/$c -o run -- \
        python3 bench.py $B1080 > gpurun_out/pmc/$c.json 2> gpurun_out/pmc/$c.err || exit $?
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc4k/$c -o run -- \
        python3 bench.py --config 4k --streams 2 --frames 12 --steps 6 --warmup 2 --no-cpu --ivf-frames 0 --output-steps 0 --prime-steps 1 > gpurun_out/pmc4k/$c.json 2> gpurun_out/pmc4k/$c.err || exit $?
done
python3 tools/pmc_traffic.py gpurun_out/pmc gpurun_out/traffic.json 8 1080p > /dev/null || exit $?
python3 tools/pmc_traffic.py gpurun_out/pmc4k gpurun_out/traffic_4k.json 2 4k > /dev/null || exit $?
bash tools/gpu_evidence_r05.sh > /dev/null || exit $?
timeout -k 10 600 python3 bench.py --traffic gpurun_out/traffic.json --traffic-4k gpurun_out/traffic_4k.json > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 --traffic gpurun_out/traffic.json > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || exit $?
find gpurun_out/prof -name "*kernel_stats.csv"
cat gpurun_out/pmcsq/report.txt
cat gpurun_out/bench.json
