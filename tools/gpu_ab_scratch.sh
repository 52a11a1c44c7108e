# A/B of the scratch fixes: the -m gpu suite on the default build, then for the default
# library and the AV1R_INTER_WAVES=3 build (k_inter without spills) a bench line and PMC
# FETCH/WRITE passes.  Every GPU step time-limited; the first failure ends the call.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    > gpurun_out/ab/gputest.log 2>&1 || { tail -40 gpurun_out/ab/gputest.log; exit 1; }
tail -2 gpurun_out/ab/gputest.log
for v in default inter3; do
    lib=av1dec_amd/_build/libav1r.so
    [ $v = inter3 ] && lib=av1dec_amd/_build/libinter3.so
    AV1R_LIB=$lib timeout -k 10 400 python3 bench.py --no-cpu > gpurun_out/ab/bench_$v.json 2> gpurun_out/ab/bench_$v.err || exit 1
    for c in FETCH_SIZE WRITE_SIZE; do
        AV1R_LIB=$lib timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/ab/pmc_$v/$c -o run -- \
            python3 bench.py --steps 8 --warmup 2 --frames 12 --no-cpu > gpurun_out/ab/pmc_$v_$c.json 2> gpurun_out/ab/pmc_$v_$c.err || exit 1
    done
    python3 tools/pmc_traffic.py gpurun_out/ab/pmc_$v gpurun_out/ab/traffic_$v.json 8 > /dev/null || exit 1
done
for v in default inter3; do echo $v; cat gpurun_out/ab/bench_$v.json; cat gpurun_out/ab/traffic_$v.json | head -12; done
