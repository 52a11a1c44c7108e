# k_flow workgroups per CU of the pipeline's solo (key) frames (AV1R_SOLO_PER_CU, default 1)
# after the flow_grid cache fix; bench without CPU / IVF / 4K / delivery legs.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/solo
for cfg in "X=0" "AV1R_SOLO_PER_CU=2" "AV1R_SOLO_PER_CU=3" "X=0" "AV1R_SOLO_PER_CU=2"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --no-4k --output-steps 0 > gpurun_out/solo/b.json 2> gpurun_out/solo/b.err || { tail -5 gpurun_out/solo/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/solo/b.json')); print('$cfg', d['value'], d['device_only_fps'])"
done
