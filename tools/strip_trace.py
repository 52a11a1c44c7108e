#!/usr/bin/env python3
"""k_strip timeline of one synthetic 1080p key frame (-DAV1R_TRACE build): per item the
phases (entry, residual, cross-strip wait, edges, predict, store, publish) and, per strip,
the time between groups.  Run on the GPU box after building the trace library here:
  python -c "from av1dec_amd import native; native.build(out='av1dec_amd/_build/libav1r_trace.so', defines=['AV1R_TRACE'])"
  python3 tools/strip_trace.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))


def main():
    path = "/tmp/strip_trace.bin"
    if os.path.exists(path):
        os.remove(path)
    os.environ["AV1R_TRACE_FILE"] = path
    os.environ.setdefault("AV1R_LIB", os.path.join(ROOT, "av1dec_amd", "_build", "libav1r_trace.so"))
    import pysynth
    from av1dec_amd import Decoder
    frames = pysynth.stream(1920, 1080, 1, 0x5EED1000, sb128=True)
    d = Decoder(0, keep_stages=False)
    d.set_discard_output(True)
    h = d.prepare(frames[0])
    d.decode_prepared(h)
    d.synchronize()
    sz0 = os.path.getsize(path)
    d.decode_prepared(h)  # the measured run (warm)
    d.synchronize()
    d.close()
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 16).astype(np.int64)[sz0 // 128:]
    a = a[a[:, 2] != 0]
    code, misc = a[:, 0], a[:, 1]
    kind = code >> 30
    txs = (misc >> 8) & 0xff
    us = lambda x: x / 100.0
    t2, t3, t4, t5, t8, t9, t10 = (a[:, i] for i in (2, 3, 4, 5, 8, 9, 10))
    f0 = t2.min()
    print(f"{len(a)} items; span {us(t5.max() - f0):.1f} us")
    # lean small-intra items (intra_fast.h): 4 wait done, 8 edges in LDS, 12 edge pass, 13
    # upsampling + DC, 9 predicted, 10 stored
    t12, t13 = a[:, 12], a[:, 13]
    ml = (kind == 0) & (t8 > 0) & (t12 > 0) & (t13 > 0) & (t9 > 0)
    for ts in np.unique(txs[ml]):
        mm = ml & (txs == ts)
        if mm.sum() < 100:
            continue
        q = lambda x, y: np.percentile(us(x[mm] - y[mm]), 50)
        print(f"  lean tx {ts:2d} n={mm.sum():6d} gather {q(t8, t4):.2f} edge pass {q(t12, t8):.2f} up+dc {q(t13, t12):.2f} "
              f"predict {q(t9, t13):.2f} store {q(t10, t9):.2f} publish {q(t5, t10):.2f}")
    m = (kind == 0) & (t8 > 0)
    for ts in np.unique(txs[m]):
        mm = m & (txs == ts)
        if mm.sum() < 100:
            continue
        q = lambda x, y: np.percentile(us(x[mm] - y[mm]), [50, 90])
        print(f"  tx {ts:2d} n={mm.sum():6d} resid %.2f/%.2f wait %.2f/%.2f edges %.2f/%.2f predict %.2f/%.2f store %.2f/%.2f publish %.2f/%.2f"
              % (*q(t3, t2), *q(t4, t3), *q(t8, t4), *q(t9, t8), *q(t10, t9), *q(t5, t10)))
    # k_flow: what paces the chain -- per level (slot 6, written by the host), the time from
    # the previous level's last store to this level's, attributed to the kind of the item
    # that stored last (its transform size; blends as -1)
    lvl = a[:, 6]
    if (lvl > 0).any() and not (a[:, 15] > 0).any():
        order = np.argsort(lvl, kind="stable")
        lv_sorted = lvl[order]
        bounds = np.flatnonzero(np.diff(lv_sorted)) + 1
        groups = np.split(order, bounds)
        prev = None
        pace = {}
        for g in groups:
            e = t10[g] if (t10[g] > 0).all() else t5[g]
            j = g[np.argmax(e)]
            end = e.max()
            if prev is not None and end > prev:
                key = -1 if kind[j] != 0 else int(txs[j])
                d = pace.setdefault(key, [0, 0.0])
                d[0] += 1
                d[1] += us(end - prev)
            prev = end if prev is None else max(prev, end)
        tot = sum(v[1] for v in pace.values())
        print(f"levels {len(groups)}; chain advance {tot / 1e3:.2f} ms, by the kind of the level's last item:")
        for key, (n, t) in sorted(pace.items(), key=lambda kv: -kv[1][1]):
            print(f"  {'blend' if key < 0 else 'tx %2d' % key}: {n:5d} levels, {t / 1e3:.3f} ms ({t / max(n, 1):.2f} us each)")
    # per strip (slot 14: strip << 32 | group, 15: the group's end after the barrier)
    strip, grp, gend = a[:, 14] >> 32, a[:, 14] & 0xffffffff, a[:, 15]
    ok = gend > 0
    print(f"rows with strip stamps: {ok.sum()} of {len(a)}")
    tot_gap = tot_work = tot_wait = 0.0
    rows = []
    for s in np.unique(strip[ok]):
        ms = ok & (strip == s)
        gs = np.unique(grp[ms])
        # per group: start = min entry, wait = max(t4 - t3), end = group end
        st = np.array([t2[ms & (grp == g)].min() for g in gs])
        en = np.array([gend[ms & (grp == g)].max() for g in gs])
        wt = np.array([us((t4 - t3)[ms & (grp == g)].max()) for g in gs])
        gap = us(st[1:] - en[:-1]) if len(gs) > 1 else np.zeros(0)
        dur = us(en - st)
        rows.append((int(s), len(gs), us(st[0] - f0), us(en[-1] - f0), dur.sum(), wt.sum(), gap.sum(), np.median(dur - wt)))
        tot_gap += gap.sum(); tot_work += (dur - wt).sum(); tot_wait += wt.sum()
    print("strip groups  start_us  end_us  sum_dur  sum_wait  sum_gap  median_group_work_us")
    for r in rows:
        print("%5d %6d %9.1f %8.1f %8.1f %8.1f %8.1f %8.2f" % r)
    print(f"total: work {tot_work / 1e3:.2f} ms, cross-strip waits {tot_wait / 1e3:.2f} ms, gaps {tot_gap / 1e3:.2f} ms")
    if ok.any():
        # the critical (last-ending) strip's groups by kind: large TBs (a side > 16, the
        # whole workgroup on the generic path), inter-intra blends, small TBs (one per wave)
        TXW = [4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64]
        TXH = [4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16]
        crit = max(rows, key=lambda r: r[3])[0]
        ms = ok & (strip == crit)
        kinds = {"large": [], "blend": [], "small": []}
        for g in np.unique(grp[ms]):
            mg = ms & (grp == g)
            big = any(max(TXW[t], TXH[t]) > 16 for t in txs[mg])
            k = "blend" if (kind[mg] != 0).any() else "large" if big else "small"
            kinds[k].append((us(gend[mg].max() - t2[mg].min()), int(mg.sum())))
        for k, v in kinds.items():
            if v:
                d = np.array([x[0] for x in v])
                print(f"  strip {crit} {k:5s} groups {len(v):5d} items {sum(x[1] for x in v):5d} "
                      f"dur p50 {np.median(d):.2f} mean {d.mean():.2f} sum {d.sum() / 1e3:.2f} ms")
    # median group phases (large vs small): item entry -> wait done, wait -> edges, ...
    w = us(t4 - t3).sum()
    tot = us(t5 - t2).sum()
    print(f"sum of item time {tot / 1e3:.1f} ms, of which waits {w / 1e3:.1f} ms")
    ph = ok & (t8 > 0)
    print("phase p50 (us): entry->resid %.2f resid->wait %.2f wait->edges %.2f edges->pred %.2f pred->store %.2f store->pub %.2f pub->groupend %.2f"
          % tuple(np.median(us(x[ph] - y[ph])) for x, y in ((t3, t2), (t4, t3), (t8, t4), (t9, t8), (t10, t9), (t5, t10), (gend, t5))))
    t11, t12 = a[:, 11], a[:, 12]
    for ts in (0, 1, 5, 6):
        m = ok & (t8 > 0) & (t11 > 0) & (txs == ts)
        md = m & (t12 > 0)  # directional modes (edge preparation stamped)
        if not m.any():
            continue
        q = lambda x, y, mm: np.median(us(x[mm] - y[mm])) if mm.any() else float("nan")
        print(f"  tx {ts:2d}: edge loads {q(t11, t4, m):.2f} edge assembly {q(t8, t11, m):.2f} | directional n={md.sum()}: "
              f"edge prep {q(t12, t8, md):.2f} predict loop {q(t9, t12, md):.2f} | other modes predict {q(t9, t8, m & ~md):.2f}")
        t13 = a[:, 13]
        me = md & (t13 > 0)
        print(f"        edge prep split: params + corner copy {q(t13, t8, me):.2f}, filter + upsample {q(t12, t13, me):.2f}")


if __name__ == "__main__":
    main()
