# round 3: the new GPU tests (headline paths, writer streams incl. hidden frames, Yami resend)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_headline.py tests/test_bsw.py tests/test_yami.py -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/gputest_r03a.log 2>&1 || { tail -60 gpurun_out/gputest_r03a.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/gputest_r03a.log | tail -40
