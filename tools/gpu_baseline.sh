cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gputest.log 2>&1 || { tail -60 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench20.json 2> gpurun_out/bench20.err || { tail -20 gpurun_out/bench20.err; exit 1; }
cat gpurun_out/bench20.json
