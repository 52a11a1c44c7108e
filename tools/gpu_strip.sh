# k_strip bring-up: key-frame time k_flow vs k_strip, the strip timeline, then the strip
# parity tests and the synthetic-stream GPU tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/keyframe_time.py 10 > gpurun_out/keyframe.txt 2>&1 || { cat gpurun_out/keyframe.txt; exit 1; }
cat gpurun_out/keyframe.txt
timeout -k 10 120 python3 -u tools/strip_trace.py > gpurun_out/strip_trace.txt 2>&1 || { cat gpurun_out/strip_trace.txt; exit 1; }
tail -22 gpurun_out/strip_trace.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k strip -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gputest_strip.log 2>&1 || { tail -40 gpurun_out/gputest_strip.log; exit 1; }
tail -2 gpurun_out/gputest_strip.log
timeout -k 10 600 python -u -m pytest tests/test_synth.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gputest_synth.log 2>&1 || { tail -40 gpurun_out/gputest_synth.log; exit 1; }
tail -2 gpurun_out/gputest_synth.log
