# GPU suite, then tools/gpu_ab_env.sh over the variants given as arguments
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { tail -40 gpurun_out/pytest.log; exit 1; }
tail -2 gpurun_out/pytest.log
bash tools/gpu_ab_env.sh "$@"
