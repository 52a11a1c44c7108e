# HBM-side traffic per stage kernel: rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in
# separate runs, kernel dispatch counters only -- no tracing domains mixed in), each GPU
# step time-limited.  Summaries land in gpurun_out/pmc/; tools/pmc_traffic.py folds them.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 900 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc/$c -o run -- \
        python3 bench.py --steps 8 --warmup 2 --frames 12 --no-cpu > gpurun_out/pmc/$c.json 2> gpurun_out/pmc/$c.err
    rc=$?
    echo "$c rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
done
find gpurun_out/pmc -name "*counter_collection*"
