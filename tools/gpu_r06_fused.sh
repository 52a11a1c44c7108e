# Round 6: the stripe-persistent fused filter kernel (k_stripe,
# -DAV1R_FUSED_STRIPE build libav1r_fused.so): final-output parity on the 172 conformance
# streams (level schedule, no stage snapshots), the 12 writer configurations (reference MD5s)
# and the headline pipeline, then the 1080p A/B against the stage kernels.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
AV1R_LIB=$PWD/av1dec_amd/_build/libav1r_fused.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_bsw.py tests/test_headline.py -m gpu -q -x -k "level_schedule or gpu_matches_reference_md5 or cycle_path" --timeout 300 --timeout-method thread > gpurun_out/fused.log 2>&1
rc=$?
tail -15 gpurun_out/fused.log
[ $rc = 0 ] || exit $rc
bash tools/gpu_r06_ab.sh --no-suite --quick av1dec_amd/_build/libav1r_fused.so
