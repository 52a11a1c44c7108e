# A/B by kernel time: rocprofv3 kernel stats of the current build and of an alternative
# libav1r.so (AV1R_LIB), twice each, same box.  usage: bash tools/ab_prof.sh other.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abprof
export TMPDIR=/tmp
ALT=$1; shift
for i in 1 2; do
    for v in cur alt; do
        if [ $v = alt ]; then export AV1R_LIB=$ALT; else unset AV1R_LIB; fi
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abprof/$v$i -o run -- \
            python3 bench.py --steps 60 --warmup 4 --no-cpu > gpurun_out/abprof/$v$i.json 2> gpurun_out/abprof/$v$i.err || exit $?
    done
done
unset AV1R_LIB
python3 - <<'PY'
import csv, glob
for d in sorted(glob.glob("gpurun_out/abprof/*/")):
    f = glob.glob(d + "*kernel_stats.csv")
    if not f:
        continue
    rows = {r["Name"][:10]: float(r["TotalDurationNs"]) / 1e6 for r in csv.DictReader(open(f[0]))}
    print(d.split("/")[-2], {k: round(v, 2) for k, v in sorted(rows.items()) if k.startswith("k_")})
PY
