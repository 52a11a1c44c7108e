# lean small-intra path bring-up: fast vs generic on synthetic key + inter frames, then the
# key-frame times and the parity suites
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 180 python3 -u tools/fi_diff.py 1920 1080 3 0x5EED1000 > gpurun_out/fi_diff.txt 2>&1 || { tail -40 gpurun_out/fi_diff.txt; exit 1; }
tail -40 gpurun_out/fi_diff.txt
grep -q "^identical" gpurun_out/fi_diff.txt || exit 1
timeout -k 10 120 python3 -u tools/keyframe_time.py 10 > gpurun_out/keyframe.txt 2>&1 || { cat gpurun_out/keyframe.txt; exit 1; }
cat gpurun_out/keyframe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_synth.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gputest_check.log 2>&1 || { tail -40 gpurun_out/gputest_check.log; exit 1; }
tail -2 gpurun_out/gputest_check.log
