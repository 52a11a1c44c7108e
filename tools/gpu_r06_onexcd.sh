# (AV1R_SOLO_XCD was an A/B build, removed after it: profiles/r06_ab_solo_onexcd.txt)
# Round 6: solo key frames on ONE XCD (AV1R_SOLO_XCD = workgroups per CU of that XCD; their
# hand-offs through its L2): the pipeline's parity tests with it on, then the default headline
# A/B of 0 (off) / 2 / 6, three rotations on one box.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/onexcd
export TMPDIR=/tmp
[ -n "$NOTEST" ] || AV1R_SOLO_XCD=6 timeout -k 10 400 python3 -u -m pytest tests/test_headline.py tests/test_multi.py tests/test_synth.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/onexcd/pytest.log 2>&1 || { tail -30 gpurun_out/onexcd/pytest.log; exit 1; }
[ -n "$NOTEST" ] || tail -1 gpurun_out/onexcd/pytest.log
n=0
for rep in 1 2 3; do
  for v in ${VARIANTS:-0 2 6}; do
    n=$((n+1))
    AV1R_SOLO_XCD=$v timeout -k 10 300 python3 bench.py --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
        > gpurun_out/onexcd/run$n.json 2> gpurun_out/onexcd/run$n.err || { echo "variant $v failed"; tail -5 gpurun_out/onexcd/run$n.err; exit 1; }
    python3 - "xcd=$v" gpurun_out/onexcd/run$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:8s} fps {d['value']:8.1f} dev {d['device_only_fps']:8.1f} stages {d['stage_ms_per_frame']} recon {d['recon_kernel_ms_per_frame']}")
PY
  done
done
