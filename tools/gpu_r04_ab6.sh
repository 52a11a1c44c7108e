# Frame-delivery trace on bench-like streams: kernels + memory copies + HIP API of the timed
# window, delivery off and on.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in none out; do
    mkdir -p gpurun_out/ab6/$m
    timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace --output-format csv -d gpurun_out/ab6/$m -o run -- python3 tools/out_probe.py 60 240 $m > gpurun_out/ab6/$m.log 2>&1 || { tail -5 gpurun_out/ab6/$m.log; exit 1; }
    grep -E "fps|window" gpurun_out/ab6/$m.log
done
