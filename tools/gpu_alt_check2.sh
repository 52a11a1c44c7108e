# GPU parity of each alternative libav1r.so, then the bench of the current build and the
# alternatives in rotation.  usage: bash tools/gpu_alt_check2.sh a.so b.so ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/alt
for lib in "$@"; do
  AV1R_LIB=$lib timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/alt/gputest.log 2>&1 || { echo "$lib"; tail -40 gpurun_out/alt/gputest.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/alt/gputest.log)"
done
for i in $(seq 1 ${AB_ROUNDS:-2}); do
  for lib in "" "$@"; do
    env ${lib:+AV1R_LIB=$lib} timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --ivf-frames 0 --output-steps 0 \
        > gpurun_out/alt/run.json 2> gpurun_out/alt/run.err || { tail -5 gpurun_out/alt/run.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/alt/run.json')); k=d['config_4k']; print('${lib:-current}', d['value'], d['device_only_fps'], d['recon_kernel_ms_per_frame'], d['stage_ms_per_frame'], '4k', k['fps'], k['device_only_fps'], k['recon_kernel_ms_per_frame'], k['stage_ms_per_frame'])"
  done
done
