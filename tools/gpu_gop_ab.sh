# How much the key frames cost the headline: the same bench with 60-frame GOPs (3 key frames
# in the 160 timed) and 240-frame GOPs (none), then a kernel trace of the default bench
# (per-step timeline: tools/timeline_steps.py).  Every GPU step time-limited.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gop
export TMPDIR=/tmp
for F in 60 240; do
  timeout -k 10 400 python3 bench.py --frames $F --steps 20 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
      > gpurun_out/gop/bench_$F.json 2> gpurun_out/gop/bench_$F.err || { tail -5 gpurun_out/gop/bench_$F.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/gop/bench_$F.json')); print('F=$F', d['value'], d['device_only_fps'], d['config']['timed_key_frames'], d['stage_ms_per_frame'], d['recon_kernel_ms_per_frame'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gop/trace -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 > gpurun_out/gop/trace.json 2>&1 || exit 1
f=$(find gpurun_out/gop/trace -name "*kernel_trace.csv" | head -1)
python3 tools/timeline_steps.py $f > gpurun_out/gop/timeline.txt && cat gpurun_out/gop/timeline.txt | head -60
gzip -f $f
