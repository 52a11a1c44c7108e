# Pipeline look-ahead A/B (AV1R_BENCH_DEPTH: frames packed ahead per stream): the 4K line
# (2 streams) and the 1080p line, each setting twice in rotation.  usage: bash tools/gpu_depth_ab.sh 3 8
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/depth
for i in 1 2; do
    for d in "$@"; do
        AV1R_BENCH_DEPTH=$d timeout -k 10 300 python3 bench.py --config 4k --streams 2 --frames 30 --steps 30 --warmup 6 --no-cpu \
            > gpurun_out/depth/4k_d$d.$i.json 2> gpurun_out/depth/4k_d$d.$i.err || exit $?
        AV1R_BENCH_DEPTH=$d timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 \
            > gpurun_out/depth/hd_d$d.$i.json 2> gpurun_out/depth/hd_d$d.$i.err || exit $?
        python3 -c "import json; a=json.load(open('gpurun_out/depth/4k_d$d.$i.json')); b=json.load(open('gpurun_out/depth/hd_d$d.$i.json')); print('depth $d', '4k', a['value'], a['host_profile'], '1080p', b['value'], b['host_profile'])"
    done
done
