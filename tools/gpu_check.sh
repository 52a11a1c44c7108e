cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 -p no:cacheprovider > gpurun_out/parity.log 2>&1
rc=$?
echo "parity rc=$rc"
tail -30 gpurun_out/parity.log
exit $rc
