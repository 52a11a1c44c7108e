# Round 6: the one-grid k_lr variant (-DAV1R_LR_ONEGRID, libav1r_lr1.so)
# through the stage-parity tests against the oracle / the reference hashes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
AV1R_LIB=$PWD/av1dec_amd/_build/libav1r_lr1.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_synth.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/lr1.log 2>&1
rc=$?
tail -30 gpurun_out/lr1.log
exit $rc
