# Round-2 evidence call: the -m gpu suite, then tools/gpu_evidence.sh (PMC traffic passes,
# the default bench line, a rocprofv3 kernel-trace/stats run).  First failure ends the call.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/gputest.log 2>&1 || { tail -60 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
bash tools/gpu_evidence.sh
