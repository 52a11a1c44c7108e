# Round 6: the GPU suite on the current build, then an A/B of the current libav1r.so against
# other builds (AV1R_LIB) on the 1080p x 8 bench (device-only rate and stage times, the
# variants in rotation, twice), then the LDS / occupancy SQ pass of each build, then the
# rocprofv3 kernel statistics of the current build.  Every GPU step time-limited; any failure
# ends the script.
# usage: bash tools/gpu_r06_ab.sh [--no-suite] [--quick] other.so [more.so ...]
# (--quick: the A/B runs only, no SQ pass and no kernel statistics)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab6 gpurun_out/prof
export TMPDIR=/tmp
QUICK=0
[ "$1" = "--quick" ] && { QUICK=1; shift; }
if [ "$1" = "--no-suite" ]; then shift; [ "$1" = "--quick" ] && { QUICK=1; shift; }; else
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { tail -40 gpurun_out/pytest.log; exit 1; }
tail -2 gpurun_out/pytest.log
fi
for i in 1 2; do
    v=0
    for lib in "" "$@"; do
        if [ -n "$lib" ]; then export AV1R_LIB=$lib; else unset AV1R_LIB; fi
        timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 \
            > gpurun_out/ab6/hd_v$v.$i.json 2> gpurun_out/ab6/hd_v$v.$i.err || exit $?
        python3 - "v$v ${lib:-current}" gpurun_out/ab6/hd_v$v.$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:34s} fps {d['value']:8.1f} dev {d['device_only_fps']:8.1f} stages {d['stage_ms_per_frame']} recon {d['recon_kernel_ms_per_frame']} kf {d['key_frame_alone_ms']['recon']}")
PY
        v=$((v + 1))
    done
done
[ $QUICK = 1 ] && exit 0
B1080="--steps 8 --warmup 2 --frames 60 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 --prime-steps 1"
v=0
for lib in "" "$@"; do
    if [ -n "$lib" ]; then export AV1R_LIB=$lib; else unset AV1R_LIB; fi
    timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE \
        --output-format csv -d gpurun_out/ab6/lds_v$v/g3 -o run -- python3 bench.py $B1080 > gpurun_out/ab6/lds_v$v.json 2> gpurun_out/ab6/lds_v$v.err || exit $?
    python3 tools/pmc_sq_report.py gpurun_out/ab6/lds_v$v > gpurun_out/ab6/lds_v$v.txt || exit $?
    echo "== v$v ${lib:-current}"; grep -E "k_cdef|k_inter_all|k_lr|k_flow" gpurun_out/ab6/lds_v$v.txt | head -12
    v=$((v + 1))
done
unset AV1R_LIB
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
