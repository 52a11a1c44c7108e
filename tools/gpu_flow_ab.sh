# parity (flow on, the default) + bench with flow on and off, every GPU step time-limited
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; echo "[$rc] $*" >> gpurun_out/steps.log; return $rc; }
ok_or_stop() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi; }
run 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; ok_or_stop $?
tail -2 gpurun_out/smoke.log
run 900 python -u -m pytest tests -q -m gpu -x --timeout 300 -p no:cacheprovider > gpurun_out/parity.log 2>&1; rc=$?
tail -5 gpurun_out/parity.log
ok_or_stop $rc
[ $rc -eq 0 ] || exit 1
run 300 python bench.py --no-cpu > gpurun_out/bench_flow.json 2> gpurun_out/bench_flow.err; ok_or_stop $?
AV1R_FLOW=0 run 300 python bench.py --no-cpu > gpurun_out/bench_lvl.json 2> gpurun_out/bench_lvl.err; ok_or_stop $?
cat gpurun_out/bench_flow.json gpurun_out/bench_lvl.json
