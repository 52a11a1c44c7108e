# lite-stamp timeline of a batched step of 8 x 1080p streams (key frames, then inter frames)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AV1R_LIB=$PWD/av1dec_amd/_build/libav1r_trace.so timeout -k 10 300 python3 tools/trace_run.py 3 /tmp/trace.bin 8 > gpurun_out/trace.txt 2>&1
rc=$?
rm -f /tmp/trace.bin
tail -70 gpurun_out/trace.txt
exit $rc
