# Kernel trace of the bench's headline and device-only legs (1080p x 8, no other legs), to
# compare per-kernel durations between the host-inclusive and the resident-batch paths.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/legs
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/legs/kt -o run -- python3 bench.py --steps 60 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 > gpurun_out/legs/b.json 2> gpurun_out/legs/b.err || { tail -5 gpurun_out/legs/b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/legs/b.json')); print(d['value'], d['device_only_fps'])"
