# (used for the r06 k_flow priority A/B, profiles/r06_ab_flow_prio.txt)
# Round 6: default headline (60 steps, no CPU / 4K / IVF / delivery legs) of the current
# libav1r.so against alternative builds (AV1R_LIB), rotated R times (R=${R:-3}).
# usage: bash tools/gpu_r06_libab.sh other.so [more.so ...]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/libab6
export TMPDIR=/tmp
n=0
for rep in $(seq ${R:-3}); do
    for lib in "" "$@"; do
        n=$((n + 1))
        if [ -n "$lib" ]; then export AV1R_LIB=$lib; else unset AV1R_LIB; fi
        timeout -k 10 300 python3 bench.py --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
            > gpurun_out/libab6/run$n.json 2> gpurun_out/libab6/run$n.err || { echo "${lib:-current} failed"; tail -5 gpurun_out/libab6/run$n.err; exit 1; }
        python3 - "${lib:-current}" gpurun_out/libab6/run$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1][-24:]:24s} fps {d['value']:8.1f} dev {d['device_only_fps']:8.1f} stages {d['stage_ms_per_frame']} recon {d['recon_kernel_ms_per_frame']} kf {d['key_frame_alone_ms']['recon']}")
PY
    done
done
unset AV1R_LIB
