# Existing pipeline knobs re-checked after the marker changes: stream groups
# (AV1R_PIPE_GROUPS), the full-batch wait (AV1R_PIPE_WAIT_US); bench without CPU / IVF / 4K
# / delivery legs.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/knobs
for cfg in "X=0" "AV1R_PIPE_GROUPS=2" "AV1R_PIPE_WAIT_US=100" "AV1R_PIPE_WAIT_US=600" "X=0" "AV1R_PIPE_GROUPS=2"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --no-4k --output-steps 0 > gpurun_out/knobs/b.json 2> gpurun_out/knobs/b.err || { tail -5 gpurun_out/knobs/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/knobs/b.json')); print('$cfg', d['value'], d['device_only_fps'], d['host_profile']['batches'])"
done
