# A/B of an environment switch: bench (1080p + 4K device-only and stages) with and without
# it, twice in rotation.  usage: bash tools/gpu_env_ab.sh VAR=value
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/envab
for i in 1 2; do
  for cfg in "" "$1"; do
    env $cfg timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --ivf-frames 0 --output-steps 0 \
        > gpurun_out/envab/run.json 2> gpurun_out/envab/run.err || { tail -5 gpurun_out/envab/run.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/envab/run.json')); k=d['config_4k']; print('${cfg:-default}', d['value'], d['device_only_fps'], d['recon_kernel_ms_per_frame'], '4k', k['fps'], k['device_only_fps'], k['recon_kernel_ms_per_frame'])"
  done
done
