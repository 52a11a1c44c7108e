cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench20.json 2> gpurun_out/bench20.err || { tail -30 gpurun_out/bench20.err; exit 1; }
cat gpurun_out/bench20.json
