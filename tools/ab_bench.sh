# A/B: bench the current build and an alternative build of libav1r.so (AV1R_LIB) on the
# same box, alternating cur/alt/cur/alt.  usage: bash tools/ab_bench.sh other.so [bench args]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ALT=$1; shift
for i in 1 2; do
    timeout -k 10 600 python bench.py --no-cpu "$@" > gpurun_out/ab_cur$i.json 2> gpurun_out/ab_cur$i.err || exit $?
    AV1R_LIB=$ALT timeout -k 10 600 python bench.py --no-cpu "$@" > gpurun_out/ab_alt$i.json 2> gpurun_out/ab_alt$i.err || exit $?
done
python3 - <<'PY'
import json
for n in ("cur1", "alt1", "cur2", "alt2"):
    d = json.load(open(f"gpurun_out/ab_{n}.json"))
    print(n, d["value"], d["stage_ms_per_frame"], "single", d["single_stream_fps"])
PY
