# Frame delivery A/B on bench-like streams: the read-back stream on a queue of its own
# (AV1R_OUT_CUMASK), completion by a pinned flag instead of an event (AV1R_OUT_FLAG),
# hardware queues per process; delivery off / on.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab5
for cfg in "X=none" "X=out" "AV1R_OUT_FLAG=1" "AV1R_OUT_CUMASK=1" "AV1R_OUT_CUMASK=1 AV1R_OUT_FLAG=1" "GPU_MAX_HW_QUEUES=16" "X=none"; do
    m=out; [ "$cfg" = "X=none" ] && m=none
    env AV1R_PIPE_PROF=1 $cfg timeout -k 10 200 python3 tools/out_probe.py 60 240 $m > gpurun_out/ab5/p.log 2>&1 || { tail -5 gpurun_out/ab5/p.log; exit 1; }
    echo "$cfg $m"; grep -E "fps" gpurun_out/ab5/p.log | tail -1
done
