# Round-2 evidence after the ABI v2 / scratch changes: the -m gpu suite, the host pack cost on
# the box's cores (1 and 15 threads), then tools/gpu_evidence.sh (PMC traffic passes, the
# default bench line, a rocprofv3 kernel-trace/stats run).  First failure ends the call.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    > gpurun_out/gputest.log 2>&1 || { tail -60 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 300 python3 tools/pack_prof.py --frames 48 --threads 1 > gpurun_out/pack_prof_1.json || exit 1
timeout -k 10 300 python3 tools/pack_prof.py --frames 48 --threads 15 > gpurun_out/pack_prof_15.json || exit 1
cat gpurun_out/pack_prof_1.json gpurun_out/pack_prof_15.json
bash tools/gpu_evidence.sh
