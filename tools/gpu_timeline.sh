# Per-dispatch timeline (kernels + memory copies) of a short batched bench run;
# summarised by tools/timeline_report.py
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tl
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tl -o run -- \
    python3 bench.py --steps 20 --warmup 4 --no-cpu > gpurun_out/tl/bench.json 2> gpurun_out/tl/bench.err
rc=$?
ls gpurun_out/tl
exit $rc
