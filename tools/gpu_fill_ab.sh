# Full-batch wait of the native launcher (AV1R_PIPE_WAIT_US), headline only, alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for w in 0 300 1000 0 300 1000; do
    AV1R_PIPE_WAIT_US=$w timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --steps 60 > gpurun_out/ab/f$w.json 2> gpurun_out/ab/f$w.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/f$w.json')); print('wait $w', d['value'], d['device_only_fps'], d['host_profile'])"
done
