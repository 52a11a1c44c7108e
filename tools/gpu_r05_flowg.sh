# k_flow small-item group size: GPU suite at the defaults and with every level grouped by 8
# (AV1R_FLOW_G_MIN=0, so that the small streams exercise the 8-item groups), then the bench A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { tail -40 gpurun_out/pytest.log; exit 1; }
tail -1 gpurun_out/pytest.log
AV1R_FLOW_G_MIN=0 timeout -k 10 600 python3 -u -m pytest tests/test_bsw.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_g8.log 2>&1 || { tail -40 gpurun_out/pytest_g8.log; exit 1; }
tail -1 gpurun_out/pytest_g8.log
bash tools/gpu_ab_env.sh - AV1R_FLOW_G=4 AV1R_FLOW_G=16 "AV1R_FLOW_G_MIN=64"
