# k_flow resident workgroups per CU (AV1R_FLOW_PER_CU) and the look-ahead depth
# (AV1R_BENCH_DEPTH) re-checked at the round-4 head; bench without CPU / IVF / 4K / delivery.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/knobs2
for cfg in "X=0" "AV1R_FLOW_PER_CU=4" "AV1R_FLOW_PER_CU=3" "AV1R_BENCH_DEPTH=12" "X=0" "AV1R_FLOW_PER_CU=4"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --no-4k --output-steps 0 > gpurun_out/knobs2/b.json 2> gpurun_out/knobs2/b.err || { tail -5 gpurun_out/knobs2/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/knobs2/b.json')); print('$cfg', d['value'], d['device_only_fps'], d['recon_kernel_ms_per_frame'], d['key_frame_alone_ms']['recon'])"
done
