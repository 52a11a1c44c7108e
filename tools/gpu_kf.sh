# key-frame timing only: k_flow vs k_strip on one 1080p key frame, then both lite-trace timelines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/keyframe_time.py 10 > gpurun_out/keyframe.txt 2>&1 || { cat gpurun_out/keyframe.txt; exit 1; }
cat gpurun_out/keyframe.txt
[ -n "$NO_TRACE" ] && exit 0
timeout -k 10 120 python3 -u tools/strip_trace.py > gpurun_out/flow_trace.txt 2>&1 || { cat gpurun_out/flow_trace.txt; exit 1; }
tail -10 gpurun_out/flow_trace.txt
AV1R_STRIP_LEVELS=400 timeout -k 10 120 python3 -u tools/strip_trace.py > gpurun_out/strip_trace.txt 2>&1 || { cat gpurun_out/strip_trace.txt; exit 1; }
tail -12 gpurun_out/strip_trace.txt
