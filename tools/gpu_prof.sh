# rocprofv3 kernel-trace + stats of a short bench run (time-limited)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 4 --no-cpu > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
rc=$?
echo "rc=$rc"
find gpurun_out/prof -name "*stats*" | head
exit $rc
