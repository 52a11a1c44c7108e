# Round 6: environment A/B on the default headline (60 steps; no CPU / 4K / IVF / delivery
# legs): each argument one variant's environment ("-" = defaults), R rotations (default 3).
# usage: bash tools/gpu_r06_envab.sh - "AV1R_BENCH_WORKERS=12" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/envab
export TMPDIR=/tmp
n=0
for rep in $(seq ${R:-3}); do
  for v in "$@"; do
    n=$((n+1))
    e=""; [ "$v" != "-" ] && e="$v"
    env $e timeout -k 10 300 python3 bench.py --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
        > gpurun_out/envab/run$n.json 2> gpurun_out/envab/run$n.err || { echo "variant '$v' failed"; tail -5 gpurun_out/envab/run$n.err; exit 1; }
    python3 - "$v" gpurun_out/envab/run$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
h = d.get("host_profile", {})
print(f"{sys.argv[1][:30]:30s} fps {d['value']:8.1f} dev {d['device_only_fps']:8.1f} recon {d['recon_kernel_ms_per_frame']} pack {h.get('pack_ms_per_frame')} util {h.get('producer_utilisation')} batches {h.get('batches')}")
PY
  done
done
