# Round 6: kernel trace + HIP runtime API trace of a short headline run (no counters), to
# line up the launcher's calls (stream waits, event syncs, launches) with the GPU timeline.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ht6
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/ht6 -o run -- \
    python3 bench.py --steps 20 --warmup 5 --frames 60 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 --prime-steps 1 > gpurun_out/ht6/bench.json 2> gpurun_out/ht6/bench.err || exit $?
ls -la gpurun_out/ht6
