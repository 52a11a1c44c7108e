# GPU parity of the writer's synthetic bitstreams (tests/test_bsw.py -m gpu), then the whole
# -m gpu suite.  First failure ends the call.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bsw.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_bsw.log 2>&1 || { tail -40 gpurun_out/gpu_bsw.log; exit 1; }
tail -3 gpurun_out/gpu_bsw.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
