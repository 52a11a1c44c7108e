# Host packing cost A/B (tools/pack_prof.py, 1 thread and 15) of two builds, then the
# parity suites that exercise the schedule (conformance stages, packed / native pipelines).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for i in 1 2; do
    for L in libold.so libav1r.so; do
        for t in 1 15; do
            echo -n "$L threads $t: "
            AV1R_LIB=av1dec_amd/_build/$L timeout -k 10 120 python3 tools/pack_prof.py --frames 48 --threads $t | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['wall_ms_per_frame'], d['cpu_ms_per_frame'], d['phase_ms_per_frame'])" || exit 1
        done
    done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "test_gpu_matches_reference or native or packed or synth" > gpurun_out/ab/parity.log 2>&1 || { tail -30 gpurun_out/ab/parity.log; exit 1; }
tail -1 gpurun_out/ab/parity.log
timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --steps 60 > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/ab/b.json')); print(d['value'], d['device_only_fps'], d['host_profile'])"
