# The bench's 4K leg (configs[3]) with launch-completion markers off (default) and on
# (AV1R_SLOT_META=0): bench without CPU / IVF legs.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k4
for cfg in "X=0" "AV1R_SLOT_META=0" "X=0" "AV1R_SLOT_META=0"; do
    env $cfg timeout -k 10 400 python3 bench.py --no-cpu --ivf-frames 0 --output-steps 0 > gpurun_out/k4/b.json 2> gpurun_out/k4/b.err || { tail -5 gpurun_out/k4/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/k4/b.json')); k=d['config_4k']; print('$cfg', d['value'], k['fps'], k.get('device_only_fps'), k.get('host_profile'))"
done
