# (AV1R_SOLO_LANE / AV1R_SOLO_WGS were an A/B build, removed after it: profiles/r06_ab_solo_lane.txt)
# Round 6: solo lane x solo k_flow grid A/B on the default headline (60 steps), two rotations.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lane2
export TMPDIR=/tmp
AV1R_SOLO_LANE=2 AV1R_SOLO_WGS=32 timeout -k 10 300 python3 -u -m pytest tests/test_headline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lane2/pytest.log 2>&1 || { tail -30 gpurun_out/lane2/pytest.log; exit 1; }
tail -1 gpurun_out/lane2/pytest.log
n=0
for rep in 1 2; do
  for v in "0 0" "0 64" "0 32" "2 0" "2 64" "2 32" "2 16"; do
    set -- $v
    n=$((n+1))
    AV1R_SOLO_LANE=$1 AV1R_SOLO_WGS=$2 timeout -k 10 300 python3 bench.py --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
        > gpurun_out/lane2/run$n.json 2> gpurun_out/lane2/run$n.err || { echo "variant $v failed"; tail -5 gpurun_out/lane2/run$n.err; exit 1; }
    python3 - "lane=$1 wgs=$2" gpurun_out/lane2/run$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:14s} fps {d['value']:8.1f} dev {d['device_only_fps']:8.1f} stages {d['stage_ms_per_frame']} recon {d['recon_kernel_ms_per_frame']}")
PY
  done
done
