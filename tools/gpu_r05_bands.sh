# k_inter_all band-major dealing (AV1R_INTER_BANDS): inter fetch (PMC FETCH_SIZE pass per
# variant, tools/pmc_traffic.py) and the bench A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bands
export TMPDIR=/tmp
B1080="--steps 8 --warmup 2 --frames 12 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 --prime-steps 1"
for v in 1 4 16; do
    mkdir -p gpurun_out/bands/b$v
    AV1R_INTER_BANDS=$v timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/bands/b$v/FETCH_SIZE -o run -- \
        python3 bench.py $B1080 > gpurun_out/bands/b$v/FETCH_SIZE.json 2> gpurun_out/bands/b$v.err || exit $?
    AV1R_INTER_BANDS=$v timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/bands/b$v/WRITE_SIZE -o run -- \
        python3 bench.py $B1080 > gpurun_out/bands/b$v/WRITE_SIZE.json 2>> gpurun_out/bands/b$v.err || exit $?
    python3 tools/pmc_traffic.py gpurun_out/bands/b$v gpurun_out/bands/traffic_b$v.json 8 1080p > /dev/null || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/bands/traffic_b$v.json')); k=d['kernels']['k_inter_all']; print('bands $v k_inter_all fetch', k['fetch_bytes_x2'], 'write', k['write_bytes'])"
done
bash tools/gpu_ab_env.sh - AV1R_INTER_BANDS=4 AV1R_INTER_BANDS=16
