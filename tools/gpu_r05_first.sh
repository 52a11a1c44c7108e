cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { tail -30 gpurun_out/pytest.log; exit 1; }
tail -3 gpurun_out/pytest.log
AV1R_LIB=$PWD/av1dec_amd/_build/libav1r_trace.so timeout -k 10 300 python3 tools/trace_run.py 3 gpurun_out/trace.bin 8 > gpurun_out/trace.txt 2>&1 || { tail -30 gpurun_out/trace.txt; exit 1; }
cat gpurun_out/trace.txt | tail -45
bash tools/gpu_evidence_r05.sh
