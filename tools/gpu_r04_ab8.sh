# Kernel / host A/B builds (AV1R_LIB): the default library against av1dec_amd/_build/exp_*.so,
# the bench's host-inclusive and device-only rates at 1080p x 8, alternated.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab8
for v in ${VARIANTS:-default exp_ring4 exp_ring6 default exp_ring4 exp_ring6}; do
    lib=""; [ $v != default ] && lib="AV1R_LIB=$GRAFT_REPO_ROOT/av1dec_amd/_build/$v.so"
    env $lib timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --no-4k ${BARGS:---output-steps 0} > gpurun_out/ab8/b.json 2> gpurun_out/ab8/b.err || { tail -5 gpurun_out/ab8/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab8/b.json')); o=d.get('output_inclusive') or {}; print('$v', d['value'], d['device_only_fps'], o.get('fps'), d['host_profile']['launcher_submit_ms_per_step'], d['stage_ms_per_frame'])"
done
