#!/usr/bin/env python3
"""One batched bench step from a rocprofv3 kernel + memory-copy trace (tools/gpu_timeline.sh):
every dispatch / copy with its start, end and the gap before it.
usage: python tools/timeline_report.py gpurun_out/tl"""
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tl"
K = list(csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])))
M = list(csv.DictReader(open(glob.glob(d + "/*memory_copy_trace.csv")[0])))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:14],
       int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])) for r in K]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r["Direction"].split("_")[-1][:6], 0) for r in M]
ev.sort()
gmax = max(e[3] for e in ev if e[2].startswith("k_inter"))
idx = [i for i, e in enumerate(ev) if e[2].startswith("k_inter") and e[3] > gmax * 0.5]
print("batched steps:", len(idx))
spans = [(ev[b][0] - ev[a][0]) / 1000 for a, b in zip(idx[:-1], idx[1:])]
print("step spans (us): median %.1f" % sorted(spans)[len(spans) // 2])
i0, i1 = idx[len(idx) // 2], idx[len(idx) // 2 + 1]
t0 = ev[i0][0]
prev_end = ev[i0 - 1][1]
busy = 0
for e in ev[i0:i1]:
    print(f"{(e[0] - t0) / 1000:9.1f} {(e[1] - t0) / 1000:9.1f}  dur {(e[1] - e[0]) / 1000:8.1f}  gap {(e[0] - prev_end) / 1000:7.1f}  {e[2]}")
    prev_end = max(prev_end, e[1])
    busy += e[1] - e[0]
print(f"step {(ev[i1][0] - t0) / 1000:.1f} us, busy {busy / 1000:.1f} us")
