# k_post (fused filters) bring-up: the paths without stage snapshots run it
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "level_schedule" -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gputest_post.log 2>&1 || { tail -40 gpurun_out/gputest_post.log; exit 1; }
tail -2 gpurun_out/gputest_post.log
timeout -k 10 900 python -u -m pytest tests/test_bsw.py tests/test_headline.py tests/test_synth.py -m gpu -x -q --timeout 600 --timeout-method thread \
    > gpurun_out/gputest_post2.log 2>&1 || { tail -40 gpurun_out/gputest_post2.log; exit 1; }
tail -2 gpurun_out/gputest_post2.log
