# fused filters (k_post) against the three stage kernels: bench stage times, then kernel stats
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/post_ab
export TMPDIR=/tmp
for f in 0 1 0 1; do
  AV1R_FUSED=$f timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
      > gpurun_out/post_ab/bench_$f.json 2> gpurun_out/post_ab/bench_$f.err || { tail -5 gpurun_out/post_ab/bench_$f.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/post_ab/bench_$f.json')); s=d['stage_ms_per_frame']; print('fused=$f', d['value'], d['device_only_fps'], s, 'filters', round(s['lf']+s['cdef']+s['lr'],4))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/post_ab/prof -o run -- \
    python3 bench.py --steps 30 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 > /dev/null 2>&1 || exit 1
f=$(find gpurun_out/post_ab/prof -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/post_ab/kernel_stats.csv; head -20 $f
