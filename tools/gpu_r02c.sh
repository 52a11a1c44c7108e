# Round-2 evidence after the bitstream writer / IVF pipeline / Yami API: the whole -m gpu
# suite, the 4K bench line (configs[3]), then tools/gpu_evidence.sh (PMC traffic passes, the
# default bench line with the IVF end-to-end leg, a rocprofv3 kernel-trace/stats run).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    > gpurun_out/gputest.log 2>&1 || { tail -60 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 600 python3 bench.py --config 4k --streams 2 --frames 30 --steps 30 --warmup 6 --no-cpu \
    > gpurun_out/bench_4k.json 2> gpurun_out/bench_4k.err || { tail -20 gpurun_out/bench_4k.err; exit 1; }
cat gpurun_out/bench_4k.json
bash tools/gpu_evidence.sh
