# GPU suite, then the batched-step trace and an A/B of the round-5 kernel switches
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { tail -40 gpurun_out/pytest.log; exit 1; }
tail -2 gpurun_out/pytest.log
bash tools/gpu_r05_trace.sh > /dev/null || exit 1
tail -60 gpurun_out/trace.txt
bash tools/gpu_ab_env.sh - AV1R_INTER_MERGED=0 AV1R_DEBLOCK_TILE=0
