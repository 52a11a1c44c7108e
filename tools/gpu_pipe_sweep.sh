# host-inclusive headline against the pipeline knobs (fill wait, look-ahead), twice each
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
for i in 1 2; do
  for cfg in "default" "AV1R_PIPE_WAIT_US=600" "AV1R_PIPE_WAIT_US=100" "AV1R_BENCH_DEPTH=12" "AV1R_BENCH_DEPTH=5"; do
    env $( [ "$cfg" = default ] || echo "$cfg" ) timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
        > gpurun_out/sweep/run.json 2> gpurun_out/sweep/run.err || { tail -5 gpurun_out/sweep/run.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/sweep/run.json')); h=d['host_profile']; print('$cfg', d['value'], d['device_only_fps'], h['batches'], h['producer_utilisation'])"
  done
done
