# SQ counter passes over one 1080p key frame on k_strip and on k_flow (instruction mix and
# where the wave cycles go: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/kfpmc
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
for k in k_strip k_flow; do
  i=1
  for P in "$P1" "$P2"; do
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/kfpmc/${k}_$i -o pmc --output-format csv -- python3 tools/keyframe_time.py 3 $k > gpurun_out/kfpmc/${k}_$i.log 2>&1 || { tail -5 gpurun_out/kfpmc/${k}_$i.log; exit 1; }
    i=$((i+1))
  done
done
ls -R gpurun_out/kfpmc | head -30
