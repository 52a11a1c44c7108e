# Stream groups interleaved (AV1R_PIPE_INTERLEAVE=1: leads on different hardware queues)
# against contiguous; bench without CPU / IVF / 4K / delivery legs, alternated.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/inter
for cfg in "X=0" "AV1R_PIPE_INTERLEAVE=1" "X=0" "AV1R_PIPE_INTERLEAVE=1"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --no-4k --output-steps 0 > gpurun_out/inter/b.json 2> gpurun_out/inter/b.err || { tail -5 gpurun_out/inter/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/inter/b.json')); print('$cfg', d['value'], d['device_only_fps'], d['host_profile']['batches'])"
done
