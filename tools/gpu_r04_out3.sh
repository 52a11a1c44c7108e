# Frame delivery at the default settings: the output GPU tests, then the bench's delivery
# leg three times (no other legs).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/out3
timeout -k 10 600 python3 -u -m pytest tests/test_headline.py -m gpu -x -v --timeout 500 --timeout-method thread -k "async or ring" -p no:cacheprovider > gpurun_out/out3/tests.log 2>&1 || { tail -30 gpurun_out/out3/tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/out3/tests.log | tail -2
bash tools/gpu_r04_out.sh
