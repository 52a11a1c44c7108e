# GPU validation + bench + profile in one gpurun call (every GPU step time-limited).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; echo "[$rc] $*" >> gpurun_out/steps.log; return $rc; }
ok_or_stop() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi; }
run 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; ok_or_stop $?
run 900 python -m pytest tests -q -m gpu -x --timeout 300 -p no:cacheprovider > gpurun_out/parity.log 2>&1; ok_or_stop $?
tail -3 gpurun_out/parity.log
run 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; ok_or_stop $?
cat gpurun_out/bench.json
