cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/strip_trace.py > gpurun_out/strip_trace.txt 2>&1; rc=$?
cat gpurun_out/strip_trace.txt
exit $rc
