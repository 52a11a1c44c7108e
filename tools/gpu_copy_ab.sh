# A/B of the packed-upload copy streams (bench headline): the batch lead's copy stream
# against every member's own, then the default bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AV1R_COPY_SPREAD=0 timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench_spread0.json 2> gpurun_out/bench_spread0.err || exit 1
AV1R_COPY_SPREAD=1 timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench_spread1.json 2> gpurun_out/bench_spread1.err || exit 1
for f in gpurun_out/bench_spread0.json gpurun_out/bench_spread1.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['device_only_fps'])"; done
