# Upload / metadata ring depth (AV1R_RING build) x frames packed ahead (AV1R_BENCH_DEPTH).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
run() {  # lib depth tag
    AV1R_LIB=av1dec_amd/_build/$1 AV1R_BENCH_DEPTH=$2 timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --steps 60 \
        > gpurun_out/ab/$3.json 2> gpurun_out/ab/$3.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$3.json')); print('$3', d['value'], d['device_only_fps'], d['host_profile'])"
}
run libav1r.so 3 r3d3
run libring6.so 3 r6d3
run libring6.so 6 r6d6
run libav1r.so 3 r3d3b
run libring6.so 6 r6d6b
