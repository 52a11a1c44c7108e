# Mode-aware intra edge dependencies (AV1R_MODE_EDGES): the -m gpu suite with them on, then
# the bench key-frame line on / off, then tools/gpu_gop_ab.sh.  Every GPU step time-limited.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/me
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
for m in 1 0; do
  AV1R_MODE_EDGES=$m timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
      > gpurun_out/me/bench_$m.json 2> gpurun_out/me/bench_$m.err || { tail -5 gpurun_out/me/bench_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/me/bench_$m.json')); print('mode_edges=$m', d['value'], d['device_only_fps'], d['key_frame_alone_ms'], d['recon_kernel_ms_per_frame'], d['recon_levels_last_frame'])"
done
bash tools/gpu_gop_ab.sh
