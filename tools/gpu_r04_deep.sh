# k_flow workgroups per CU for a deep frame launched by itself (AV1R_DEEP_PER_CU): the
# bench's key-frame-alone time and rates (no CPU / IVF / 4K / delivery legs).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/deep
for cfg in "X=0" "AV1R_DEEP_PER_CU=3" "AV1R_DEEP_PER_CU=2" "AV1R_DEEP_PER_CU=4" "X=0" "AV1R_DEEP_PER_CU=3"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --no-4k --output-steps 0 > gpurun_out/deep/b.json 2> gpurun_out/deep/b.err || { tail -5 gpurun_out/deep/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/deep/b.json')); print('$cfg', d['value'], d['device_only_fps'], d['key_frame_alone_ms'])"
done
