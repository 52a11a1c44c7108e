# A/B of HBM traffic per stage: PMC passes (FETCH_SIZE, WRITE_SIZE) of the current build and
# of an alternative libav1r.so (AV1R_LIB), each folded by tools/pmc_traffic.py, then the
# kernel-time A/B (tools/ab_prof.sh).  usage: bash tools/gpu_traffic_ab.sh other.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tab
export TMPDIR=/tmp
for v in cur alt; do
    mkdir -p gpurun_out/tab/$v
    if [ $v = alt ]; then export AV1R_LIB=$1; else unset AV1R_LIB; fi
    for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/tab/$v/$c -o run -- \
            python3 bench.py --steps 8 --warmup 2 --frames 12 --no-cpu > gpurun_out/tab/$v/$c.json 2> gpurun_out/tab/$v/$c.err || exit $?
    done
    python3 tools/pmc_traffic.py gpurun_out/tab/$v gpurun_out/tab/traffic_$v.json 8 > /dev/null || exit $?
    echo "== $v"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['stages'])" gpurun_out/tab/traffic_$v.json
done
unset AV1R_LIB
bash tools/ab_prof.sh "$@"
