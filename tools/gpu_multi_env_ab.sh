# A/B of several environment settings against the default, in rotation (twice), 1080p bench
# (host-inclusive, device-only, recon kernels, key frame).  usage: bash tools/gpu_multi_env_ab.sh "A=1" "B=2 C=3" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/menv
for i in 1 2; do
  for cfg in "" "$@"; do
    env $cfg timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
        > gpurun_out/menv/run.json 2> gpurun_out/menv/run.err || { tail -5 gpurun_out/menv/run.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/menv/run.json')); print('${cfg:-default}', d['value'], d['device_only_fps'], d['recon_kernel_ms_per_frame'], d['stage_ms_per_frame'], d['key_frame_alone_ms']['recon'])"
  done
done
