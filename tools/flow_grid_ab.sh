# A/B of k_flow's resident workgroups per CU (AV1R_FLOW_PER_CU), bench k_flow ms/frame
cd $GRAFT_REPO_ROOT
for r in 1 2; do for p in 4 3 2; do
  AV1R_FLOW_PER_CU=$p timeout -k 10 300 python bench.py --no-cpu > gpurun_out/fg_$p.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/fg_$p.json')); print('per_cu $p', d['value'], d['recon_kernel_ms_per_frame'], d['single_stream_fps'])"
done; done
