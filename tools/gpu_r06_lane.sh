# (AV1R_SOLO_LANE / AV1R_SOLO_WGS were an A/B build, removed after it: profiles/r06_ab_solo_lane.txt)
# Round 6: the solo lane A/B (AV1R_SOLO_LANE 0 / 1 / 2) on the default headline (60 steps),
# three rotations on one box, after the headline parity tests with the low-priority lane.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lane
export TMPDIR=/tmp
AV1R_SOLO_LANE=1 timeout -k 10 300 python3 -u -m pytest tests/test_headline.py tests/test_multi.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lane/pytest.log 2>&1 || { tail -30 gpurun_out/lane/pytest.log; exit 1; }
tail -1 gpurun_out/lane/pytest.log
n=0
for rep in 1 2 3; do
  for v in 0 1 2; do
    n=$((n+1))
    AV1R_SOLO_LANE=$v timeout -k 10 300 python3 bench.py --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
        > gpurun_out/lane/run$n.json 2> gpurun_out/lane/run$n.err || { echo "variant $v failed"; tail -5 gpurun_out/lane/run$n.err; exit 1; }
    python3 - "lane=$v" gpurun_out/lane/run$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:10s} fps {d['value']:8.1f} dev {d['device_only_fps']:8.1f} stages {d['stage_ms_per_frame']} recon {d['recon_kernel_ms_per_frame']}")
PY
  done
done
