# Round evidence at the current head in one call: the -m gpu suite, the 4K line (configs[3]),
# then tools/gpu_evidence.sh
# (PMC traffic passes, the default bench line reading that traffic, rocprofv3 kernel stats).
# AV1R_GIT_HEAD (the commit measured) is set by the caller.  Every GPU step time-limited.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 600 python3 bench.py --config 4k --streams 2 --frames 30 --steps 30 --warmup 6 --no-cpu \
    > gpurun_out/bench_4k.json 2> gpurun_out/bench_4k.err || { tail -20 gpurun_out/bench_4k.err; exit 1; }
bash tools/gpu_evidence.sh
