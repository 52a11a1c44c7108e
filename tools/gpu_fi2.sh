# lean-path change: A/B against the generic path, key frames, lean-path timeline, parity
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 180 python3 -u tools/fi_diff.py 1920 1080 3 0x5EED1000 > gpurun_out/fi_diff.txt 2>&1 || { tail -40 gpurun_out/fi_diff.txt; exit 1; }
tail -3 gpurun_out/fi_diff.txt
grep -q "^identical" gpurun_out/fi_diff.txt || exit 1
timeout -k 10 120 python3 -u tools/keyframe_time.py 10 > gpurun_out/keyframe.txt 2>&1 || { cat gpurun_out/keyframe.txt; exit 1; }
cat gpurun_out/keyframe.txt
timeout -k 10 120 python3 -u tools/strip_trace.py > gpurun_out/flow_trace.txt 2>&1 || { cat gpurun_out/flow_trace.txt; exit 1; }
head -9 gpurun_out/flow_trace.txt; grep -A12 "^levels" gpurun_out/flow_trace.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_synth.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gputest_check.log 2>&1 || { tail -40 gpurun_out/gputest_check.log; exit 1; }
tail -2 gpurun_out/gputest_check.log
