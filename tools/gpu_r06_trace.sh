# Round 6: the lite-stamp timeline of a batched step of 8 x 1080p streams (tools/trace_run.py,
# -DAV1R_TRACE -DAV1R_TRACE_LITE build), then the A/B of the given builds (gpu_r06_ab.sh, no suite).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AV1R_LIB=$PWD/av1dec_amd/_build/libav1r_trace.so timeout -k 10 300 python3 tools/trace_run.py 3 /tmp/trace.bin 8 > gpurun_out/trace.txt 2>&1 || { tail -30 gpurun_out/trace.txt; exit 1; }
rm -f /tmp/trace.bin
tail -80 gpurun_out/trace.txt
[ $# -gt 0 ] && bash tools/gpu_r06_ab.sh --no-suite "$@"
