# Round-3 evidence at the current tree in one call: the -m gpu suite, then
# tools/gpu_evidence_r03.sh (PMC traffic at 1080p and 4K, the bench line reading it, a
# rocprofv3 kernel-trace/stats run of the same bench).  AV1R_GIT_HEAD set by the caller.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
bash tools/gpu_evidence_r03.sh
