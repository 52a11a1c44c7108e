# Round 6: the host-to-device upload's share of the headline -- kernel and memory-copy
# traces of the 1080p x 8 bench (headline + device-only legs), with statistics.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/copy6
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/copy6 -o run -- \
    python3 bench.py --steps 30 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 > gpurun_out/copy6/bench.json 2> gpurun_out/copy6/bench.err || exit $?
find gpurun_out/copy6 -name "*stats.csv" | while read f; do echo "== $f"; head -8 "$f"; done
