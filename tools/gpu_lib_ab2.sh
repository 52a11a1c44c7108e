# GPU parity of the current build, then the bench of the current build and of an
# alternative libav1r.so (AV1R_LIB) in rotation.  usage: bash tools/gpu_lib_ab2.sh other.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
for i in 1 2; do
  for lib in "" "$1"; do
    env ${lib:+AV1R_LIB=$lib} timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --ivf-frames 0 --output-steps 0 \
        > gpurun_out/ab2/run.json 2> gpurun_out/ab2/run.err || { tail -5 gpurun_out/ab2/run.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab2/run.json')); k=d['config_4k']; print('${lib:-current}', d['value'], d['device_only_fps'], d['recon_kernel_ms_per_frame'], d['key_frame_alone_ms']['recon'], '4k', k['fps'], k['device_only_fps'], k['recon_kernel_ms_per_frame'])"
  done
done
