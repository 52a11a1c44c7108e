# WRITE_SIZE / FETCH_SIZE per kernel and frame for the current build and alternatives (AV1R_LIB),
# then the kernel-time A/B.  usage: bash tools/gpu_ab_traffic.sh other.so [...]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abtr
export TMPDIR=/tmp
v=0
for lib in "" "$@"; do
    if [ -n "$lib" ]; then export AV1R_LIB=$lib; else unset AV1R_LIB; fi
    for c in WRITE_SIZE FETCH_SIZE; do
        timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/abtr/v$v/$c -o run -- \
            python3 bench.py --steps 8 --warmup 2 --frames 12 --no-cpu > /dev/null 2> gpurun_out/abtr/v$v.$c.err || exit $?
    done
    python3 - gpurun_out/abtr/v$v "$lib" <<'PY'
import csv, glob, sys
from collections import defaultdict
d, lib = sys.argv[1], sys.argv[2] or "current"
out = []
for c in ("WRITE_SIZE", "FETCH_SIZE"):
    tot = defaultdict(float)
    nf = 0
    for f in glob.glob(d + "/" + c + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != c:
                continue
            k = r["Kernel_Name"].split("(")[0]
            tot[k] += float(r["Counter_Value"]) * 1024
            if k == "k_cdef":
                nf += 1
    out.append(c + " MB/launch " + str({k: round(v / max(nf, 1) / 1e6, 1) for k, v in sorted(tot.items()) if k.startswith("k_")}))
print(lib, *out)
PY
    v=$((v + 1))
done
unset AV1R_LIB
bash tools/ab_prof.sh "$@"
