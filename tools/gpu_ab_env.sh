# A/B of environment switches on the 1080p x 8 bench (no CPU / 4K / IVF / delivery legs):
# each argument is one variant's environment ("-" = defaults), run in turn, twice.
# usage: bash tools/gpu_ab_env.sh - "AV1R_X=0" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
n=0
for rep in 1 2; do
  for v in "$@"; do
    n=$((n+1))
    e=""; [ "$v" != "-" ] && e="$v"
    env $e timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
        > gpurun_out/ab/run$n.json 2> gpurun_out/ab/run$n.err || { echo "variant '$v' failed"; tail -5 gpurun_out/ab/run$n.err; exit 1; }
    python3 - "$v" gpurun_out/ab/run$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:28s} fps {d['value']:8.1f} dev {d['device_only_fps']:8.1f} stages {d['stage_ms_per_frame']} recon {d['recon_kernel_ms_per_frame']} kf {d['key_frame_alone_ms']['recon']}")
PY
  done
done
