# bench fps under several environment settings (same build), twice each in rotation
# usage: [BENCH_ARGS="--steps 20 --warmup 5"] bash tools/gpu_envab.sh "AV1R_SPLIT=1" "AV1R_SPLIT=2" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/envab
for i in 1 2; do
    v=0
    for e in "$@"; do
        env $e timeout -k 10 300 python3 bench.py --no-cpu $BENCH_ARGS > gpurun_out/envab/v$v.$i.json 2> gpurun_out/envab/v$v.$i.err || exit $?
        python3 -c "import json,sys; d=json.load(open('gpurun_out/envab/v$v.$i.json')); print('$e', d['value'], d.get('device_only_fps'), d['stage_ms_per_frame'], d['single_stream_fps'])"
        v=$((v + 1))
    done
done
