# GPU parity of the current build, then rocprof kernel totals of current vs an alternative
# libav1r.so (tools/ab_prof.sh).  usage: bash tools/gpu_ab.sh av1dec_amd/_build/other.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 -p no:cacheprovider > gpurun_out/parity.log 2>&1
rc=$?
tail -3 gpurun_out/parity.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_prof.sh "$@"
