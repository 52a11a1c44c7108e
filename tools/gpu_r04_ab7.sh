# Frame delivery A/B on bench-like streams: read-backs on the context's upload stream
# (AV1R_OUT_ON_COPY) against their own stream; stream groups.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab7
for cfg in "X=none" "X=out" "AV1R_OUT_ON_COPY=1" "X=out" "AV1R_OUT_ON_COPY=1" "AV1R_OUT_ON_COPY=1 AV1R_PIPE_GROUPS=2" "AV1R_PIPE_GROUPS=2"; do
    m=out; [ "$cfg" = "X=none" ] && m=none
    env $cfg timeout -k 10 200 python3 tools/out_probe.py 60 240 $m > gpurun_out/ab7/p.log 2>&1 || { tail -5 gpurun_out/ab7/p.log; exit 1; }
    echo "$cfg $m"; grep -E "fps" gpurun_out/ab7/p.log | tail -1
done
