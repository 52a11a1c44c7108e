# Frame delivery: the output GPU tests, then delivery off / on (read-backs on the upload
# stream, one linear copy per frame into the ring sink's device-layout slots) / on with a
# read-back stream of its own (AV1R_OUT_ON_COPY=0), then the bench's legs.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab5
timeout -k 10 600 python3 -u -m pytest tests/test_headline.py -m gpu -x -v --timeout 500 --timeout-method thread -k "async or ring" -p no:cacheprovider > gpurun_out/ab5/tests.log 2>&1 || { tail -30 gpurun_out/ab5/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/ab5/tests.log | tail -5
for cfg in "X=none" "X=out" "AV1R_OUT_ON_COPY=0" "X=out" "AV1R_OUT_ON_COPY=0"; do
    m=out; [ "$cfg" = "X=none" ] && m=none
    env $cfg timeout -k 10 200 python3 tools/out_probe.py 60 240 $m > gpurun_out/ab5/p.log 2>&1 || { tail -5 gpurun_out/ab5/p.log; exit 1; }
    echo "$cfg $m"; grep -E "fps" gpurun_out/ab5/p.log | tail -1
done
timeout -k 10 300 python3 bench.py --steps 60 --warmup 5 --no-cpu --ivf-frames 0 --no-4k --output-steps 120 > gpurun_out/ab5/run.json 2> gpurun_out/ab5/run.err || { tail -5 gpurun_out/ab5/run.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab5/run.json')); o=d['output_inclusive']; print(d['value'], d['host_profile']); print('  out', {k: v for k, v in o.items() if k != 'method'})"
