# Two stream groups by default from 8 streams: the bench (no CPU / IVF legs; 1080p, 4K and
# delivery) at the default and with one group (AV1R_PIPE_GROUPS=1), alternated.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/groups
for cfg in "X=0" "AV1R_PIPE_GROUPS=1" "X=0" "AV1R_PIPE_GROUPS=1"; do
    env $cfg timeout -k 10 400 python3 bench.py --no-cpu --ivf-frames 0 > gpurun_out/groups/b.json 2> gpurun_out/groups/b.err || { tail -5 gpurun_out/groups/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/groups/b.json')); o=d['output_inclusive']; print('$cfg', d['value'], d['device_only_fps'], o['fps'], o['vs_headline'], d['config_4k']['fps'])"
done
