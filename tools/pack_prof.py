#!/usr/bin/env python3
"""Host cost of the pipeline's per-frame work (av1r_pack: validation, dependency schedule,
packing copy), by phase, on the bench's synthetic 1080p streams.  Host only (no device
needed; pinned memory when one is present).

    AV1R_PACK_PROF=1 python tools/pack_prof.py [--frames 48] [--threads 1]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))
os.environ.setdefault("AV1R_PACK_PROF", "1")

PHASES = ["validate", "sched_init", "sched_blocks", "sched_items", "sched_deps", "copy"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=48)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import bench
    from av1dec_amd import Decoder, native
    l = native.lib()
    frames = bench.rank_streams("1080p", 0, 1, a.frames)[0][1:]  # the inter frames
    ns = (C.c_uint64 * 7)()
    best = None
    for _ in range(a.reps):
        l.av1r_pack_profile(ns, 7, 1)
        t = time.perf_counter()
        with ThreadPoolExecutor(a.threads) as ex:
            ps = list(ex.map(Decoder.pack, frames))
        wall = time.perf_counter() - t
        l.av1r_pack_profile(ns, 7, 0)
        packed = sum(l.av1r_packed_bytes(p) for p in ps) / max(len(ps), 1)
        for p in ps:
            Decoder.free_packed(p)
        n = max(int(ns[6]), 1)
        r = {"threads": a.threads, "frames": len(frames), "wall_ms_per_frame": round(1e3 * wall / len(frames), 3),
             "phase_ms_per_frame": {ph: round(ns[i] / n / 1e6, 3) for i, ph in enumerate(PHASES)},
             "packed_MB_per_frame": round(packed / 1e6, 3)}
        r["cpu_ms_per_frame"] = round(sum(r["phase_ms_per_frame"].values()), 3)
        if best is None or r["cpu_ms_per_frame"] < best["cpu_ms_per_frame"]:
            best = r
    print(json.dumps(best))


if __name__ == "__main__":
    main()
