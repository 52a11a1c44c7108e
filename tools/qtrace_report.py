#!/usr/bin/env python3
"""The stream -> hardware-queue map of a headline run, and the GPU timeline around every
key frame launched alone (tools/gpu_r06_qtrace.sh: rocprofv3 --kernel-trace
--memory-copy-trace).  rocprofv3's kernel trace names each dispatch's HSA queue (Queue_Id)
and HIP stream (Stream_Id): the runtime maps GPU_MAX_HW_QUEUES (4) queues to all streams,
so this shows which streams share one in-order queue.

usage: python tools/qtrace_report.py gpurun_out/qt6 [window_ms]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/qt6"
kf = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
mf = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)
ev = []
qmap = defaultdict(set)
for r in csv.DictReader(open(kf[0])):
    s, q = r.get("Stream_Id", "?"), r.get("Queue_Id", "?")
    qmap[s].add(q)
    y = r.get("Grid_Size_Y", r.get("Grid_Size", "?"))
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:12], s, q, y))
for f in mf:
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")[-6:],
                   r.get("Stream_Id", "?"), "sdma", ""))
ev.sort()
t0 = ev[0][0]
print("stream -> queue(s):")
for s in sorted(qmap, key=lambda x: int(x) if x.isdigit() else 1 << 30):
    print(f"  stream {s:>4}: queue {' '.join(sorted(qmap[s]))}")
solo = [e for e in ev if e[2].startswith("k_flow") and e[1] - e[0] > 1_000_000]
print(f"{len(solo)} k_flow dispatches over 1 ms")
win = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 0.4e6
for k, e in enumerate(solo[:3]):
    print(f"--- solo k_flow {k}: {(e[0] - t0) / 1e6:.3f}-{(e[1] - t0) / 1e6:.3f} ms, stream {e[3]} queue {e[4]}")
    for x in ev:
        if e[0] - 2 * win <= x[0] <= e[1] + win:
            print(f"  {(x[0] - t0) / 1e6:10.3f}-{(x[1] - t0) / 1e6:10.3f} ms  {x[2]:14s} stream {x[3]:>4} queue {x[4]:>6} {x[5]}")
# how much of the run no batch kernel was running (gaps between kernels of other streams)
busy = []
for x in ev:
    if x[4] != "sdma":
        busy.append((x[0], x[1]))
busy.sort()
gap, end = 0, busy[0][1]
for a, b in busy[1:]:
    if a > end:
        gap += a - end
    end = max(end, b)
print(f"GPU kernel-idle time: {gap / 1e6:.3f} ms of {(end - busy[0][0]) / 1e6:.3f} ms")
