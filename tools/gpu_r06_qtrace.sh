# Round 6: kernel + memory-copy trace of a short headline run (no counters): the stream ->
# HSA queue map (Queue_Id) and the timeline around each key frame launched alone.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qt6
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/qt6 -o run -- \
    python3 bench.py --steps 20 --warmup 5 --frames 60 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 --prime-steps 1 > gpurun_out/qt6/bench.json 2> gpurun_out/qt6/bench.err || exit $?
python3 tools/qtrace_report.py gpurun_out/qt6 > gpurun_out/qt6/report.txt || exit $?
head -80 gpurun_out/qt6/report.txt
