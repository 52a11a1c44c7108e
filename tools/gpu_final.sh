# Round evidence at the current head in one call: the -m gpu suite, then tools/gpu_evidence.sh
# (PMC traffic passes, the default bench line reading that traffic, rocprofv3 kernel stats).
# AV1R_GIT_HEAD (the commit measured) is set by the caller.  Every GPU step time-limited.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
bash tools/gpu_evidence.sh
