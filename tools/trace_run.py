#!/usr/bin/env python3
"""Per-item timeline of the recon kernels (debug): decodes a few frames of one synthetic
stream with AV1R_TRACE_FILE set and summarises where each work item's time goes.
Run on the GPU box:  python3 tools/trace_run.py [frames] [out.bin]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))


def run(nfr, path, streams=1):
    if os.path.exists(path):
        os.remove(path)
    os.environ["AV1R_TRACE_FILE"] = path
    # the timeline needs the -DAV1R_TRACE build (av1dec_amd.native.build(out=..., defines=["AV1R_TRACE"]))
    os.environ.setdefault("AV1R_LIB", os.path.join(ROOT, "av1dec_amd", "_build", "libav1r_trace.so"))
    import pysynth
    from av1dec_amd import Decoder
    decs, hss = [], []
    for i in range(streams):
        frames = pysynth.stream(1920, 1080, nfr, 0x5EED1000 + i, sb128=True)
        d = Decoder(0, keep_stages=False)
        d.set_discard_output(True)
        decs.append(d)
        hss.append([d.prepare(f) for f in frames])
    sizes = [0]
    for t in range(nfr):
        if streams == 1:
            decs[0].decode_prepared(hss[0][t])
        else:
            Decoder.decode_prepared_batch(decs, [h[t] for h in hss])
        for d in decs:
            d.synchronize()
        sizes.append(os.path.getsize(path))
    for d in decs:
        d.close()
    return sizes


def summarise(path):
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 16).astype(np.int64)
    code, misc, t0, t1, t2, t3, lvl = a[:, 0], a[:, 1], a[:, 2], a[:, 3], a[:, 4], a[:, 5], a[:, 6]
    kind = code >> 30
    pred = misc & 0xff
    txs = (misc >> 8) & 0xff
    # frames: level index resets to 0
    starts = np.flatnonzero((lvl == 0) & np.r_[True, lvl[1:] != lvl[:-1]][: len(lvl)])
    print(f"{len(a)} items, {len(starts)} frame(s)")
    us = lambda x: x / 100.0  # 100 MHz counter -> us
    for name, m in (("TB intra", (kind == 0) & (pred == 0)), ("TB inter", (kind == 0) & (pred == 2)),
                    ("inter tile", kind == 1), ("ii blend", kind == 2)):
        if not m.any():
            continue
        d_item = us(t1[m] - t0[m]); d_pred = us(np.where(kind[m] == 0, t2[m] - t1[m], 0)); d_all = us(t3[m] - t0[m])
        print(f"{name:11s} n={m.sum():7d}  item-load p50 {np.median(d_item):6.2f}  pred p50 {np.median(d_pred):6.2f}"
              f"  total p50 {np.median(d_all):6.2f} p90 {np.percentile(d_all, 90):6.2f} max {d_all.max():7.2f} us")
    # inter tiles by motion mode / compound: setup+plane-0 prediction, plane 0 total, rest
    m = kind == 1
    t7 = a[:, 7]
    mm_mode = (misc >> 16) & 0xf
    comp = (misc >> 20) & 1
    for mode in np.unique(mm_mode[m]):
        for cp in (0, 1):
            mm = m & (mm_mode == mode) & (comp == cp)
            if not mm.any():
                continue
            print(f"   inter tile motion {mode} compound {cp}: n={mm.sum():6d} item {np.median(us(t1[mm]-t0[mm])):5.2f}"
                  f" luma-pred {np.median(us(t2[mm]-t1[mm])):5.2f} luma-store {np.median(us(t7[mm]-t2[mm])):5.2f}"
                  f" chroma {np.median(us(t3[mm]-t7[mm])):5.2f} total {np.median(us(t3[mm]-t0[mm])):5.2f}")
    # sub-phases of intra TBs (small mode: 4x4, 8x8, 16x16)
    for ts in (0, 1, 2, 3):
        mm = (kind == 0) & (pred == 0) & (txs == ts) & (a[:, 8] > 0) & (a[:, 13] > 0)
        if not mm.any():
            continue
        ph = lambda i, j: np.median(us(a[mm, j] - a[mm, i]))
        print(f"   intra tx {ts}: item {ph(2,3):.2f} edges {ph(3,8):.2f} predict {ph(8,9):.2f} cfl/sync {ph(9,4):.2f}"
              f" zero {ph(4,11):.2f} dequant {ph(11,12):.2f} rows {ph(12,13):.2f} cols+store {ph(13,5):.2f}")
    # per tx size, intra TBs
    m = (kind == 0) & (pred == 0)
    for ts in np.unique(txs[m]):
        mm = m & (txs == ts)
        print(f"   intra tx_size {ts:2d}: n={mm.sum():6d} total p50 {np.median(us(t3[mm]-t0[mm])):6.2f} pred {np.median(us(t2[mm]-t1[mm])):6.2f} resid {np.median(us(t3[mm]-t2[mm])):6.2f}")
    for fi in sorted({0, len(starts) - 1}):
        level_report(a, starts, fi)


def level_report(a, starts, fi):
    import collections
    code, misc, t0, t3, lvl = a[:, 0], a[:, 1], a[:, 2], a[:, 5], a[:, 6]
    kind = code >> 30
    txs = (misc >> 8) & 0xff
    us = lambda x: x / 100.0
    f0 = starts[fi]
    f1 = starts[fi + 1] if fi + 1 < len(starts) else len(a)
    sl = slice(f0, f1)
    L = lvl[sl]
    ul = np.unique(L)
    spans = [us(t3[sl][L == l].max() - t0[sl][L == l].min()) for l in ul]
    gaps = [us(t0[sl][L == l2].min() - t3[sl][L == l1].max()) for l1, l2 in zip(ul[:-1], ul[1:])]
    print(f"frame {fi}: levels {len(ul)}, sum of level spans {sum(spans):.1f} us, sum of gaps {sum(gaps):.1f} us"
          f" (median gap {np.median(gaps) if gaps else 0:.2f})")
    names = {0: "TB", 1: "tile", 2: "ii"}
    rows = []
    for l in ul:
        mm = np.flatnonzero(L == l)
        ends = t3[sl][mm]
        j = mm[np.argmax(ends)]
        rows.append((l, len(mm), names[int(kind[sl][j])], int(txs[sl][j]), us(t3[sl][j] - t0[sl][j]),
                     np.median(us(t3[sl][mm] - t0[sl][mm])), us(ends.max() - t0[sl][mm].min())))
    print("level  items straggler(kind,tx) dur  median  span")
    for r in rows[:10] + rows[-4:]:
        print("%5d %6d %6s %3d %7.2f %7.2f %7.2f" % r)
    c = collections.Counter((r[2], r[3]) for r in rows)
    print("stragglers by (kind, tx_size):", c.most_common(8))
    # span histogram
    sp = np.array(spans)
    print("level span percentiles (us): p10 %.1f p50 %.1f p90 %.1f max %.1f" % tuple(np.percentile(sp, [10, 50, 90, 100])))


def summarise_flow(path, lo=0, hi=None):
    """k_flow-mode timeline (frame-major rows): per item entry (2), residual done (3),
    dependencies complete (4), published (5); inter tiles (k_inter) stamp 2, 3, 5."""
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 16).astype(np.int64)
    a = a[lo // 128: (hi // 128 if hi else None)]
    a = a[a[:, 2] != 0]  # rows of items that did not run in this mode (inter TBs: k_resid)
    code, misc, t2, t3, t4, t5, lvl, x7 = (a[:, i] for i in (0, 1, 2, 3, 4, 5, 6, 7))
    kind = code >> 30
    pred = misc & 0xff
    txs = (misc >> 8) & 0xff
    us = lambda x: x / 100.0
    flow = kind != 1
    tiles = kind == 1
    t0 = t2[tiles].min() if tiles.any() else t2[flow].min()
    print(f"{len(a)} items: {tiles.sum()} inter tiles, {flow.sum()} flow items")
    if tiles.any():
        print(f"k_inter: first entry 0, last end {us(t5[tiles].max() - t0):.1f} us; tile p50 {np.median(us(t5[tiles]-t2[tiles])):.2f} us")
        bs = misc & 0xff
        mm_ = (misc >> 8) & 0xf
        cp = (misc >> 12) & 1
        t8, t9, t10, t11, t12 = (a[:, i] for i in (8, 9, 10, 11, 12))
        names = ["4x4", "4x8", "8x4", "8x8", "8x16", "16x8", "16x16", "16x32", "32x16", "32x32", "32x64", "64x32",
                 "64x64", "64x128", "128x64", "128x128", "4x16", "16x4", "8x32", "32x8", "16x64", "64x16"]
        print("  tile class            n   entry->item  item->geo  geo->lumapred  ->luma-store  ->U  ->V  total (us, p50)")
        for b_ in np.unique(bs[tiles]):
            for mo in np.unique(mm_[tiles]):
                for c_ in (0, 1):
                    m = tiles & (bs == b_) & (mm_ == mo) & (cp == c_)
                    if m.sum() < 50:
                        continue
                    med = lambda x, y: np.median(us(x[m] - y[m]))
                    print(f"  {names[b_]:7s} motion {mo} comp {c_} {m.sum():6d}   {med(t3, t2):6.2f}  {med(t11, t3):6.2f}"
                          f"  {med(t12, t11):6.2f}  {med(t8, t12):6.2f}  {med(t9, t8):6.2f}  {med(t10, t9):6.2f}  {med(t5, t2):6.2f}")
    f0 = t2[flow].min()
    print(f"k_flow: first entry {us(f0 - t0):.1f} us, last publish {us(t5[flow].max() - t0):.1f} us (span {us(t5[flow].max() - f0):.1f})")
    for name, m in (("TB intra", flow & (kind == 0) & (pred == 0)), ("TB palette", flow & (kind == 0) & (pred == 1)),
                    ("TB inter", flow & (kind == 0) & (pred == 2)), ("ii blend", kind == 2), ("intra blk", kind == 3)):
        if not m.any():
            continue
        r = us(t3[m] - t2[m]); w = us(t4[m] - t3[m]); f = us(t5[m] - t4[m])
        print(f"{name:10s} n={m.sum():7d} resid p50 {np.median(r):5.2f} wait p50 {np.median(w):6.2f} p90 {np.percentile(w, 90):7.2f}"
              f" finish p50 {np.median(f):5.2f} p90 {np.percentile(f, 90):5.2f}  last publish {us(t5[m].max() - t0):8.1f} us")
    m = flow & (kind == 0) & (pred == 0) & (a[:, 8] > 0)
    if m.any():  # granule build: 8 edges gathered, 9 predicted, 10 stored + granules out
        t8, t9, t10 = a[:, 8], a[:, 9], a[:, 10]
        for ts in np.unique(txs[m]):
            mm = m & (txs == ts)
            if mm.sum() < 200:
                continue
            q = lambda x, y: np.percentile(us(x[mm] - y[mm]), [50, 90])
            print(f"   intra tx {ts:2d}: gather(wait) p50/p90 %.2f/%.2f  predict %.2f/%.2f  store %.2f/%.2f  publish %.2f/%.2f"
                  % (*q(t8, t4), *q(t9, t8), *q(t10, t9), *q(t5, t10)))
    m = flow & (kind == 0) & (pred == 0)
    for ts in np.unique(txs[m]):
        mm = m & (txs == ts)
        print(f"   intra tx {ts:2d}: n={mm.sum():6d} resid {np.median(us(t3[mm]-t2[mm])):5.2f} finish {np.median(us(t5[mm]-t4[mm])):5.2f}"
              f" finish p90 {np.percentile(us(t5[mm]-t4[mm]), 90):5.2f}")
    # busy vs waiting items over time (10 us buckets)
    end = t5[flow].max()
    edges = np.arange(f0, end + 1000, 1000)
    def active(s_, e_):
        c = np.zeros(len(edges) - 1)
        for lo, hi in zip(s_, e_):
            i0 = np.searchsorted(edges, lo, "right") - 1
            i1 = np.searchsorted(edges, hi, "right") - 1
            c[max(i0, 0):i1 + 1] += 1
        return c
    wait = active(t3[flow], t4[flow])
    work = active(t2[flow], t3[flow]) + active(t4[flow], t5[flow])
    print("10-us buckets of k_flow: items waiting / working (every 10th bucket)")
    for i in range(0, len(wait), max(1, len(wait) // 25)):
        print(f"  t={us(edges[i] - f0):7.0f} us  waiting {wait[i]:6.0f}  working {work[i]:6.0f}")


def summarise_slots(path, lo=0, hi=None):
    """Where a batched k_flow launch's wave-time goes (lite timeline: every stamp is the time the
    wave REACHED that point).  Per wave slot (HW_ID + XCC id of stamp 7) the items it ran in
    entry order; the launch span split, summed over slots, into: between items (ticket atomic,
    group load, the group's barrier: the slowest of the group's four items), setup (record,
    block, residual prefetch, fi_setup: 2 -> 3), dependency wait (3 -> 4), edge gather incl.
    granule polls (4 -> 8), prediction (8 -> 9), store (9 -> 10), publish (10 -> 5)."""
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 16).astype(np.int64)
    a = a[lo // 128: (hi // 128 if hi else None)]
    code = a[:, 0]
    kind = code >> 30
    a = a[(a[:, 2] != 0) & (kind != 1)]
    if not len(a):
        return
    t2, t3, t4, t5, t8, t9, t10 = (a[:, i] for i in (2, 3, 4, 5, 8, 9, 10))
    x7 = a[:, 7].astype(np.uint64)
    slot = (x7 >> np.uint64(16))  # HW_ID << 16 | XCC
    us = lambda x: x / 100.0
    span = t5.max() - t2.min()
    slots = np.unique(slot)
    between = 0
    gaps = []
    for s_ in slots:
        m = np.flatnonzero(slot == s_)
        o = m[np.argsort(t2[m])]
        g = t2[o[1:]] - t5[o[:-1]]
        gaps.append(g)
        between += g.clip(min=0).sum()
    gaps = np.concatenate(gaps) if gaps else np.zeros(1)
    have = (t4 <= t8) & (t8 <= t9) & (t9 <= t10) & (t10 <= t5)  # the lean path's stamps (others: stale)
    tot = len(slots) * span
    parts = {"setup 2->3": (t3 - t2).sum(), "dep wait 3->4": (t4 - t3).sum(),
             "gather 4->8": np.where(have, t8 - t4, 0).sum(), "predict 8->9": np.where(have, t9 - t8, 0).sum(),
             "store 9->10": np.where(have, t10 - t9, 0).sum(), "publish 10->5": np.where(have, t5 - t10, 0).sum(),
             "other paths 4->5": np.where(have, 0, t5 - t4).sum(), "between items": between}
    print(f"k_flow slots: {len(slots)} wave slots seen, {len(a)} items ({len(a) / len(slots):.1f} per slot), "
          f"span {us(span):.1f} us; per item p50 {np.median(us(t5 - t2)):.2f} us, gap between a slot's items "
          f"p50 {np.median(us(gaps)):.2f} p90 {np.percentile(us(gaps), 90):.2f} us")
    for k, v in parts.items():
        print(f"   {k:18s} {v / tot:6.1%} of slot-time  ({us(v) / len(a):6.2f} us per item)")
    print(f"   {'idle (after last)':18s} {1 - sum(parts.values()) / tot:6.1%}")
    # the chain: per dependency level, when its items start, are released and finish
    lvl = a[:, 6]
    base = t2.min()
    print("level  items  start p10/p50  released p50/p90  end p50/p90/max (us from the launch's first item)")
    for l in np.unique(lvl):
        m = lvl == l
        q = lambda x, p: np.percentile(us(x[m] - base), p)
        print(f"{l:5d} {m.sum():6d}   {q(t2, 10):7.1f} {q(t2, 50):7.1f}   {q(t4, 50):7.1f} {q(t4, 90):7.1f}"
              f"   {q(t5, 50):7.1f} {q(t5, 90):7.1f} {q(t5, 100):7.1f}")


if __name__ == "__main__":
    nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "trace.bin")
    streams = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    os.makedirs(os.path.dirname(path), exist_ok=True)
    sizes = run(nfr, path, streams)
    if os.environ.get("AV1R_FLOW", "1") != "0":
        print("=== first step (key frames) ===")
        summarise_flow(path, sizes[0], sizes[1])
        print("=== last step ===")
        summarise_flow(path, sizes[-2], sizes[-1])
        summarise_slots(path, sizes[-2], sizes[-1])
    else:
        summarise(path)
