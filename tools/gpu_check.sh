# quick GPU check after a kernel change: key-frame time (k_flow, k_strip), the parity
# suite of the conformance + synthetic streams, the k_flow / k_strip item timelines
# (lite trace library), a 20-step bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_synth.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gputest_check.log 2>&1 || { tail -40 gpurun_out/gputest_check.log; exit 1; }
tail -2 gpurun_out/gputest_check.log
timeout -k 10 120 python3 -u tools/keyframe_time.py 10 > gpurun_out/keyframe.txt 2>&1 || { cat gpurun_out/keyframe.txt; exit 1; }
cat gpurun_out/keyframe.txt
timeout -k 10 120 python3 -u tools/strip_trace.py > gpurun_out/flow_trace.txt 2>&1 || { cat gpurun_out/flow_trace.txt; exit 1; }
tail -12 gpurun_out/flow_trace.txt
AV1R_STRIP_LEVELS=400 timeout -k 10 120 python3 -u tools/strip_trace.py > gpurun_out/strip_trace.txt 2>&1 || { cat gpurun_out/strip_trace.txt; exit 1; }
tail -12 gpurun_out/strip_trace.txt
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-4k > gpurun_out/bench20.json 2> gpurun_out/bench20.err || { tail -20 gpurun_out/bench20.err; exit 1; }
cat gpurun_out/bench20.json
