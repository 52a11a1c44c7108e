# One GPU call: the -m gpu suite, the k_flow overlap probe (debug + product builds), the
# default bench line.  Every GPU step time-limited; the first failure ends the call.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
    > gpurun_out/gputest.log 2>&1 || { tail -60 gpurun_out/gputest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -3 gpurun_out/gputest.log
if [ -z "$SKIP_PROBE" ]; then bash tools/flow_overlap_probe.sh || exit 1; fi
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
