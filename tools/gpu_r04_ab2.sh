# Round-4 A/Bs after the suite passed: k_flow per-wave items, inter tiles by reference, and
# the frame-delivery leg (AV1R_OUT_NOCOPY: the machinery without the copies).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab2
for i in 1 2; do
  for cfg in "" "AV1R_FLOW_WAVE=1" "AV1R_INTER_ORDER=1" "AV1R_OUT_NOCOPY=1"; do
    env $cfg timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --ivf-frames 0 > gpurun_out/ab2/run.json 2> gpurun_out/ab2/run.err || { tail -5 gpurun_out/ab2/run.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab2/run.json')); k=d['config_4k']; o=d['output_inclusive']; print('${cfg:-default}', d['value'], d['device_only_fps'], d['stage_ms_per_frame'], d['recon_kernel_ms_per_frame'], 'kf', d['key_frame_alone_ms']['recon'], 'out', o['fps'], '4k', k['fps'], k['device_only_fps'], k['recon_kernel_ms_per_frame'])"
  done
done
