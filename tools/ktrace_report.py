#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (tools/gpu_trace.sh): per kernel name the dispatch
count and mean/total device time, plus k_flow dispatches split into the slow (key-frame)
and regular ones.  usage: python tools/ktrace_report.py gpurun_out/ktrace"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ktrace"
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
by = defaultdict(list)
for r in rows:
    by[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
for k, v in sorted(by.items(), key=lambda kv: -sum(x[1] for x in kv[1])):
    tot = sum(x[1] for x in v)
    print(f"{k[:40]:40s} n={len(v):6d} total={tot / 1e6:9.2f} ms mean={tot / len(v) / 1e3:9.1f} us max={max(x[1] for x in v) / 1e3:9.1f} us")
fl = sorted(x[1] for x in by.get("k_flow", []))
if fl:
    med = fl[len(fl) // 2]
    slow = [x for x in fl if x > 4 * med]
    fast = [x for x in fl if x <= 4 * med]
    print(f"k_flow: median {med / 1e3:.1f} us; {len(slow)} slow dispatches mean {sum(slow) / max(len(slow), 1) / 1e3:.1f} us; "
          f"{len(fast)} regular mean {sum(fast) / max(len(fast), 1) / 1e3:.1f} us")
