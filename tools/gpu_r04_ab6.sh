# Frame-delivery trace on bench-like streams: kernels + memory copies of the timed window,
# read-backs by k_out (default) and by the copy engine.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in kout sdma; do
    mkdir -p gpurun_out/ab6/$m
    sd=0; [ $m = sdma ] && sd=1
    AV1R_OUT_SDMA=$sd timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/ab6/$m -o run -- python3 tools/out_probe.py 60 240 out > gpurun_out/ab6/$m.log 2>&1 || { tail -5 gpurun_out/ab6/$m.log; exit 1; }
    grep -E "fps|window" gpurun_out/ab6/$m.log
done
