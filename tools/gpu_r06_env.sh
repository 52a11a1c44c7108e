# Round 6: environment A/B of the 1080p x 8 headline (tools/gpu_ab_env.sh's loop, 60 timed
# steps as the default bench): each argument is one variant's environment ("-" = defaults).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/env6
n=0
for rep in 1 2; do
  for v in "$@"; do
    n=$((n+1))
    e=""; [ "$v" != "-" ] && e="$v"
    env $e timeout -k 10 300 python3 bench.py --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
        > gpurun_out/env6/run$n.json 2> gpurun_out/env6/run$n.err || { echo "variant '$v' failed"; tail -5 gpurun_out/env6/run$n.err; exit 1; }
    python3 - "$v" gpurun_out/env6/run$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
h = d["host_profile"]
print(f"{sys.argv[1]:28s} fps {d['value']:8.1f} dev {d['device_only_fps']:8.1f} pack {h['pack_ms_per_frame']} util {h['producer_utilisation']} submit {h['launcher_submit_ms_per_step']} batches {h['batches']}")
PY
  done
done
