# The -m gpu suite, then a driver-style bench line, at the current tree.  Every GPU step
# time-limited; a failing step ends the script.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err \
    || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
