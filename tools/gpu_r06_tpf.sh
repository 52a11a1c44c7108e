# (AV1R_TINY_PREFETCH was an A/B build, removed after it: profiles/r06_ab_tiny_prefetch.txt)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gop
timeout -k 10 800 python3 -u -m pytest tests/test_multi.py -m gpu -k whole_gop -x -v -s --timeout 700 --timeout-method thread > gpurun_out/gop/pytest.log 2>&1 || { tail -20 gpurun_out/gop/pytest.log; exit 1; }
tail -3 gpurun_out/gop/pytest.log
AV1R_LIB=av1dec_amd/_build/libav1r_tpf.so timeout -k 10 300 python3 -u -m pytest tests/test_headline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gop/pytest_tpf.log 2>&1 || { tail -20 gpurun_out/gop/pytest_tpf.log; exit 1; }
tail -1 gpurun_out/gop/pytest_tpf.log
R=3 bash tools/gpu_r06_libab.sh av1dec_amd/_build/libav1r_tpf.so
