# A/B by kernel time: rocprofv3 kernel stats of the current build and of alternative
# libav1r.so builds (AV1R_LIB), twice each in rotation, same box.
# usage: bash tools/ab_prof.sh other.so [more.so ...]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abprof
export TMPDIR=/tmp
for i in 1 2; do
    v=0
    for lib in "" "$@"; do
        if [ -n "$lib" ]; then export AV1R_LIB=$lib; else unset AV1R_LIB; fi
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abprof/v$v.$i -o run -- \
            python3 bench.py --steps 60 --warmup 4 --no-cpu > gpurun_out/abprof/v$v.$i.json 2> gpurun_out/abprof/v$v.$i.err || exit $?
        v=$((v + 1))
    done
done
unset AV1R_LIB
python3 - "$@" <<'PY'
import csv, glob, json, sys
libs = ["current"] + sys.argv[1:]
for d in sorted(glob.glob("gpurun_out/abprof/v*/")):
    f = glob.glob(d + "**/*kernel_stats.csv", recursive=True)
    if not f:
        continue
    tag = d.rstrip("/").split("/")[-1]
    rows = {r["Name"][:10]: float(r["TotalDurationNs"]) / 1e6 for r in csv.DictReader(open(f[0]))}
    k = {a: round(b, 1) for a, b in sorted(rows.items()) if a.startswith("k_")}
    try:
        fps = json.load(open(d.rstrip("/") + ".json"))["value"]
    except Exception:
        fps = None
    print(tag, libs[int(tag[1:].split(".")[0])], "fps", fps, "sum", round(sum(k.values()), 1), k)
PY
