# Pack buffers: a new buffer instead of waiting for a busy one (up to a bound), the bench
# without CPU / IVF / 4K legs, twice.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/slot
for i in 1 2; do
    timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --no-4k > gpurun_out/slot/b.json 2> gpurun_out/slot/b.err || { tail -5 gpurun_out/slot/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/slot/b.json')); o=d['output_inclusive']; print(d['value'], d['device_only_fps'], o['fps'], o['vs_headline'], d['host_profile']['pack_ms_per_frame'], o['pack_ms_per_frame'])"
done
