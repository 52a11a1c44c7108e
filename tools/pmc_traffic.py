#!/usr/bin/env python3
"""Fold the rocprofv3 FETCH_SIZE / WRITE_SIZE dispatch counters of tools/gpu_pmc.sh into
per-stage bytes per frame -> profiles/traffic.json (read by bench.py as roofline.traffic).

FETCH_SIZE and WRITE_SIZE are the L2 memory-side (fabric) request bytes; Infinity-Cache
hits count as traffic.  MI355X_MICROARCH.md (HBM section): gfx950 FETCH_SIZE reports half
the bytes of wide coalesced reads, so the corrected read figure is 2x FETCH_SIZE; byte-wide
access patterns are uncalibrated -- both raw and corrected values are recorded."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

STAGES = {"k_inter": "recon", "k_inter_m": "recon", "k_inter_s": "recon", "k_inter_all": "recon", "k_tb": "recon",
          "k_resid_s": "recon", "k_resid_l": "recon", "k_flow": "recon",
          "k_mi_zero": "recon", "k_mi_blocks": "recon", "k_mi_tbs": "recon",
          "k_lf": "lf", "k_cdef": "cdef", "k_lr": "lr"}


def fold(path, counter):
    files = glob.glob(os.path.join(path, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {path}")
    tot = defaultdict(float)
    per_kernel = defaultdict(float)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].strip()
            st = STAGES.get(name)
            if st is None:
                continue
            v = float(r["Counter_Value"]) * (1024 if counter.endswith("_SIZE") else 1)
            tot[st] += v
            per_kernel[name] += v
            if st == "cdef":
                rows.append(int(r["Grid_Size"]))
    # one k_cdef launch covers every frame of its batch: frames = grid / one frame's grid
    one = min(rows) if rows else 1
    frames = sum(round(g / one) for g in rows)
    return tot, frames, per_kernel


def main():
    base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json")
    fetch, nf, fk = fold(os.path.join(base, "FETCH_SIZE"), "FETCH_SIZE")
    write, nw, wk = fold(os.path.join(base, "WRITE_SIZE"), "WRITE_SIZE")
    stages = {}
    for st in dict.fromkeys(STAGES.values()):
        f = fetch.get(st, 0.0) / max(nf, 1)
        w = write.get(st, 0.0) / max(nw, 1)
        stages[st] = {"fetch_bytes_raw": round(f), "fetch_bytes_x2": round(2 * f), "write_bytes": round(w),
                      "traffic_bytes": round(2 * f + w)}
    res = {"config": sys.argv[4] if len(sys.argv) > 4 else "1080p", "streams": int(sys.argv[3]) if len(sys.argv) > 3 else 8,
           "frames_fetch": nf, "frames_write": nw,
           "git_head": os.environ.get("AV1R_GIT_HEAD"),  # the commit the counters were collected at (no .git on the box)
           "unit": "bytes per frame (per stage, all launches of the frame)",
           "stages": {k: v["traffic_bytes"] for k, v in stages.items()}, "detail": stages,
           "kernels": {k: {"fetch_bytes_x2": round(2 * fk.get(k, 0.0) / max(nf, 1)), "write_bytes": round(wk.get(k, 0.0) / max(nw, 1))}
                       for k in sorted(set(fk) | set(wk))}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
