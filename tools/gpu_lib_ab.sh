# Stage times and device-only fps of the current libav1r.so against alternative builds
# (AV1R_LIB), at 4K (2 streams, 4x2 tiles) and 1080p (8 streams), twice each in rotation.
# usage: bash tools/gpu_lib_ab.sh other.so [more.so ...]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/libab
for i in 1 2; do
    v=0
    for lib in "" "$@"; do
        if [ -n "$lib" ]; then export AV1R_LIB=$lib; else unset AV1R_LIB; fi
        timeout -k 10 300 python3 bench.py --config 4k --streams 2 --frames 30 --steps 30 --warmup 6 --no-cpu \
            > gpurun_out/libab/4k_v$v.$i.json 2> gpurun_out/libab/4k_v$v.$i.err || exit $?
        timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 > gpurun_out/libab/hd_v$v.$i.json 2> gpurun_out/libab/hd_v$v.$i.err || exit $?
        python3 -c "import json; a=json.load(open('gpurun_out/libab/4k_v$v.$i.json')); b=json.load(open('gpurun_out/libab/hd_v$v.$i.json')); print('v$v ${lib:-current}', '4k', a['device_only_fps'], a['stage_ms_per_frame'], '1080p', b['device_only_fps'], b['stage_ms_per_frame'])"
        v=$((v + 1))
    done
done
unset AV1R_LIB
