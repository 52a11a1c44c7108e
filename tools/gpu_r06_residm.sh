# Round 6: k_resid_l with two TBs of at most 32x32 per workgroup (32 lanes each): the whole GPU
# suite with it, then the headline A/B against the previous build (libav1r_rm0.so).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rm
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/rm/pytest.log 2>&1 || { tail -40 gpurun_out/rm/pytest.log; exit 1; }
tail -1 gpurun_out/rm/pytest.log
R=3 bash tools/gpu_r06_libab.sh av1dec_amd/_build/libav1r_rm0.so
