# Kernel A/B builds (AV1R_LIB): the default library against av1dec_amd/_build/exp_*.so, the
# bench's device-only stage times at 1080p x 8, alternated.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab8
for v in default exp_cdef default exp_cdef; do
    lib=""; [ $v != default ] && lib="AV1R_LIB=$GRAFT_REPO_ROOT/av1dec_amd/_build/$v.so"
    env $lib timeout -k 10 300 python3 bench.py --steps 60 --warmup 5 --no-cpu --ivf-frames 0 --no-4k --output-steps 0 > gpurun_out/ab8/b.json 2> gpurun_out/ab8/b.err || { tail -5 gpurun_out/ab8/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab8/b.json')); print('$v', d['value'], d['device_only_fps'], d['stage_ms_per_frame'], d['recon_kernel_ms_per_frame'])"
done
