# rocprofv3 kernel trace (per dispatch) + stats of a short bench run; bench line alongside
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ktrace
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktrace -o run -- \
    python3 bench.py --steps 60 --warmup 4 --no-cpu "$@" > gpurun_out/ktrace/bench.json 2> gpurun_out/ktrace/bench.err
rc=$?
echo "rc=$rc"
cat gpurun_out/ktrace/bench.json
exit $rc
