# Launcher profile (AV1R_PIPE_PROF) of the bench-like pipeline without delivery.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pp
AV1R_PIPE_PROF=1 timeout -k 10 200 python3 tools/out_probe.py 60 240 none > gpurun_out/pp/p.log 2>&1 || { tail -5 gpurun_out/pp/p.log; exit 1; }
grep -E "fps|av1r pipe" gpurun_out/pp/p.log | tail -3
