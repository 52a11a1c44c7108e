# Launch completion through the launch's own meta event (default) against events per slot,
# per packed buffer and per status record (AV1R_SLOT_META=0): the synthetic and headline
# parity tests at the default, then the bench (no CPU / IVF / 4K legs), alternated.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/slot
timeout -k 10 600 python3 -u -m pytest tests/test_headline.py tests/test_synth.py tests/test_multi.py -m gpu -x -q --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/slot/tests.log 2>&1 || { tail -30 gpurun_out/slot/tests.log; exit 1; }
tail -1 gpurun_out/slot/tests.log
for cfg in "X=0" "AV1R_SLOT_META=0" "X=0" "AV1R_SLOT_META=0"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --no-4k > gpurun_out/slot/b.json 2> gpurun_out/slot/b.err || { tail -5 gpurun_out/slot/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/slot/b.json')); o=d['output_inclusive']; print('$cfg', d['value'], d['device_only_fps'], o['fps'], o['vs_headline'], d['host_profile']['pack_ms_per_frame'])"
done
