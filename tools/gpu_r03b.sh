# headline parity (persistent pipeline), the 20-step bench with the launcher profile, then
# device-only A/B of the current build against $1 (1080p, twice in rotation)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest tests/test_headline.py -x -q --timeout 900 --timeout-method thread > gpurun_out/headline.log 2>&1
rc=$?; tail -3 gpurun_out/headline.log; [ $rc -eq 0 ] || exit $rc
AV1R_PIPE_PROF=1 timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-4k > gpurun_out/bench20p.json 2> gpurun_out/bench20p.err || { tail -5 gpurun_out/bench20p.err; exit 1; }
grep "av1r pipe" gpurun_out/bench20p.err | tail -3
[ -n "$1" ] || exit 0
for i in 1 2; do
  for v in cur alt; do
    if [ $v = alt ]; then export AV1R_LIB=$1; else unset AV1R_LIB; fi
    timeout -k 10 300 python3 bench.py --no-cpu --no-4k --ivf-frames 0 --output-steps 0 > gpurun_out/ab/$v$i.json 2> gpurun_out/ab/$v$i.err || { tail -5 gpurun_out/ab/$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab/$v$i.json')); print('$v$i', d['value'], d['device_only_fps'], d['stage_ms_per_frame'], d['key_frame_alone_ms']['recon'])"
  done
done
