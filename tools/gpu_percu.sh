# k_flow key-frame time against the resident workgroups per CU (AV1R_FLOW_PER_CU)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 5 3 2 1; do
  echo "per CU $n"
  AV1R_FLOW_PER_CU=$n timeout -k 10 120 python3 -u tools/keyframe_time.py 10 k_flow || exit 1
done
