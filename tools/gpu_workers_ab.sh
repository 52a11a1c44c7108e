# Packing-thread count of the native pipeline (AV1R_BENCH_WORKERS) against the box's 16-CPU
# quota, headline only.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for w in 15 8 11 6 15 8; do
    AV1R_BENCH_WORKERS=$w timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --steps 60 > gpurun_out/ab/w$w.json 2> gpurun_out/ab/w$w.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/w$w.json')); print('workers $w', d['value'], d['device_only_fps'], d['host_profile'])"
done
