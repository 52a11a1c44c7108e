#!/usr/bin/env python3
"""Kernel timeline of a bench run from a rocprofv3 --kernel-trace CSV: how busy the GPU is,
how long each kernel runs while a solo key frame (a k_flow launch longer than 2 ms) runs
beside it and while none does, and the idle gaps between kernels of one queue.

    python3 tools/timeline_steps.py run_kernel_trace.csv[.gz] [--since SECONDS_FROM_END]"""
import csv
import gzip
import sys
from collections import defaultdict


def load(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        rows = list(csv.DictReader(f))
    out = []
    for r in rows:
        name = r.get("Kernel_Name", "")
        name = name.split("(")[0].strip()
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "0")))
    out.sort()
    return out


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    path = sys.argv[1]
    since = None
    if "--since" in sys.argv:
        since = float(sys.argv[sys.argv.index("--since") + 1])
    ks = load(path)
    if since is not None:
        end = max(e for _, e, _, _ in ks)
        ks = [k for k in ks if k[0] >= end - since * 1e9]
    span = max(e for _, e, _, _ in ks) - min(s for s, _, _, _ in ks)
    busy = union([(s, e) for s, e, _, _ in ks])
    keys = [(s, e) for s, e, n, _ in ks if n == "k_flow" and e - s > 2_000_000]
    key_busy = union(keys)
    print(f"kernels {len(ks)}  span {span / 1e6:.1f} ms  busy {busy / span:.3f}  solo key frames {len(keys)} "
          f"(running {key_busy / span:.3f} of the span, {sum(e - s for s, e in keys) / max(1, len(keys)) / 1e3:.0f} us avg)")
    nonkey = [(s, e) for s, e, n, _ in ks if not (n == "k_flow" and e - s > 2_000_000)]
    nk_busy = union(nonkey)
    print(f"other kernels busy {nk_busy / span:.3f} of the span")

    def overlaps(s, e):
        for a, b in keys:
            if a < e and s < b:
                return True
        return False
    stats = defaultdict(lambda: [0, 0, 0, 0])  # n with key, total with key, n without, total without
    for s, e, n, _ in ks:
        if n == "k_flow" and e - s > 2_000_000:
            continue
        st = stats[n]
        if overlaps(s, e):
            st[0] += 1
            st[1] += e - s
        else:
            st[2] += 1
            st[3] += e - s
    print(f"{'kernel':24s} {'n(key)':>7s} {'us(key)':>9s} {'n(alone)':>9s} {'us(alone)':>10s}")
    for n, (a, b, c, d) in sorted(stats.items(), key=lambda kv: -(kv[1][1] + kv[1][3])):
        print(f"{n:24s} {a:7d} {b / max(a, 1) / 1e3:9.1f} {c:9d} {d / max(c, 1) / 1e3:10.1f}")
    # idle between consecutive kernels of one queue
    byq = defaultdict(list)
    for s, e, n, q in ks:
        byq[q].append((s, e, n))
    for q, lst in sorted(byq.items()):
        gaps = [lst[i + 1][0] - lst[i][1] for i in range(len(lst) - 1)]
        gaps = [g for g in gaps if g > 0]
        if not gaps:
            continue
        gaps.sort()
        print(f"queue {q}: {len(lst)} kernels, gap median {gaps[len(gaps) // 2] / 1e3:.1f} us, "
              f"p90 {gaps[int(len(gaps) * 0.9)] / 1e3:.1f} us, total {sum(gaps) / 1e6:.1f} ms")


if __name__ == "__main__":
    main()
