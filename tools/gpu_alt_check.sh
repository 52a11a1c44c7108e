# GPU parity of an alternative libav1r.so (AV1R_LIB), then the bench of the current build and
# the alternative in rotation.  usage: bash tools/gpu_alt_check.sh alt.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/alt
AV1R_LIB=$1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/alt/gputest.log 2>&1 || { tail -40 gpurun_out/alt/gputest.log; exit 1; }
tail -2 gpurun_out/alt/gputest.log
AB_ROUNDS=${AB_ROUNDS:-2}
for i in $(seq 1 $AB_ROUNDS); do
  for lib in "" "$1"; do
    env ${lib:+AV1R_LIB=$lib} timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --ivf-frames 0 --output-steps 0 \
        > gpurun_out/alt/run.json 2> gpurun_out/alt/run.err || { tail -5 gpurun_out/alt/run.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/alt/run.json')); k=d['config_4k']; print('${lib:-current}', d['value'], d['device_only_fps'], d['recon_kernel_ms_per_frame'], '4k', k['fps'], k['device_only_fps'], k['recon_kernel_ms_per_frame'])"
  done
done
