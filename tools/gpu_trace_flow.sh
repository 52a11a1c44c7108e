# k_flow timeline of a batched key step and an inter step (8 streams), -DAV1R_TRACE build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/trace_run.py 4 /tmp/trace.bin 8 > gpurun_out/trace_flow.txt 2>&1
rc=$?
cat gpurun_out/trace_flow.txt
exit $rc
