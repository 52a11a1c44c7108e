# Round 6: instruction-cache counters per kernel (are the large kernels -- k_inter_all 135 KB,
# k_cdef 84 KB, k_flow 83 KB of code -- fetch-bound?).  Lists the SQC counters first and runs
# the pass only if they exist; one small counter set, its own time limit.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/icache
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --list-avail > gpurun_out/icache/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*\|SQC_TC_INST[A-Z_]*" gpurun_out/icache/avail.txt | sort -u > gpurun_out/icache/names.txt
cat gpurun_out/icache/names.txt
grep -q "^SQC_ICACHE_MISSES$" gpurun_out/icache/names.txt || { echo "no SQC_ICACHE_MISSES"; exit 0; }
B1080="--steps 8 --warmup 2 --frames 60 --no-cpu --no-4k --ivf-frames 0 --output-steps 0 --prime-steps 1"
timeout -s KILL 180 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES --output-format csv -d gpurun_out/icache/p1 -o run -- \
    python3 bench.py $B1080 > gpurun_out/icache/p1.json 2> gpurun_out/icache/p1.err || { tail -5 gpurun_out/icache/p1.err; exit 1; }
python3 - <<'PY'
import csv, glob
from collections import defaultdict
tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob("gpurun_out/icache/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Kernel_Name"][:16]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQC_ICACHE_REQ", 0)):
    req, miss, w = c.get("SQC_ICACHE_REQ", 0), c.get("SQC_ICACHE_MISSES", 0), c.get("SQ_WAVES", 1)
    print(f"{k:16s} waves {w:10.0f} icache req/wave {req / max(w, 1):8.1f} miss/wave {miss / max(w, 1):7.2f} miss rate {miss / max(req, 1):.3f}")
PY
