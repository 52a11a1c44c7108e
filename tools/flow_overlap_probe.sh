# Probe: the threaded stress (8 contexts, 8 host threads, no serial first
# frame) on the -DAV1R_FLOW_DEBUG build, which counts k_flow workgroup entries that find
# another launch's workgroups still running and how many such pairs came from different
# streams; the product build's run must show no k_flow wait timeout either
cd $GRAFT_REPO_ROOT
AV1R_LIB=av1dec_amd/_build/libflowdbg.so timeout -k 10 300 python tools/thr_stress.py 3 > gpurun_out/ov_dbg.txt 2>&1 || exit $?
timeout -k 10 300 python tools/thr_stress.py 3 > gpurun_out/ov_prod.txt 2>&1 || exit $?
cat gpurun_out/ov_dbg.txt gpurun_out/ov_prod.txt
