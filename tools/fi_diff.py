#!/usr/bin/env python3
"""A/B of the lean small-intra path (av1r_set_fast_intra): decode synthetic frames with it
on and off, compare the reconstruction (stage 0) and report, per plane, the mismatching
pixels and the transform blocks that contain them (mode, size, position).
usage (GPU box): python3 tools/fi_diff.py [width height frames seed]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))


# Tx_Width / Tx_Height by TX_SIZE (TX_4X4 .. TX_64X16)
TX_W = [4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64]
TX_H = [4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16]


def recon(frames, fast):
    from av1dec_amd import Decoder, native
    native.lib().av1r_set_fast_intra(fast)
    d = Decoder(0, keep_stages=True)
    out = []
    for f in frames:
        d.decode_frame(f)
        out.append([p.copy() for p in d.read_stage(0)])
        while d.output_pending():
            d.get_output()
    d.close()
    return out


def main():
    w, h, n, seed = (int(a, 0) for a in (sys.argv[1:5] if len(sys.argv) > 4 else ("1920", "1080", "2", "0x5EED1000")))
    import pysynth
    from av1dec_amd import abi
    frames = pysynth.stream(w, h, n, seed, sb128=True)
    a = recon(frames, 1)
    b = recon(frames, 0)
    bad = 0
    for fi, (fa, fb) in enumerate(zip(a, b)):
        tbs = np.frombuffer(frames[fi].sec["tbs"].tobytes(), dtype=abi.TB_DTYPE)
        blks = np.frombuffer(frames[fi].sec["blocks"].tobytes(), dtype=abi.BLOCK_DTYPE)
        for p, (pa, pb) in enumerate(zip(fa, fb)):
            ys, xs = np.nonzero(pa != pb)
            if not len(ys):
                continue
            bad += len(ys)
            print(f"frame {fi} plane {p}: {len(ys)} pixels differ")
            sel = tbs[tbs["plane"] == p]
            seen = set()
            for y, x in zip(ys, xs):
                m = (sel["x"] <= x) & (sel["y"] <= y)
                cand = sel[m]
                if not len(cand):
                    continue
                # the TB containing (x, y): the last one in decode order starting at or before it
                for t in cand[::-1]:
                    tw, th = TX_W[t["tx_size"]], TX_H[t["tx_size"]]
                    if x < t["x"] + tw and y < t["y"] + th:
                        key = (int(t["x"]), int(t["y"]))
                        if key not in seen:
                            seen.add(key)
                            bk = blks[t["block"]]
                            print(f"  tb at ({t['x']},{t['y']}) tx {t['tx_size']} ({tw}x{th}) flags {t['flags']} "
                                  f"y_mode {bk['y_mode']} uv_mode {bk['uv_mode']} ad {bk['angle_delta_y']}/{bk['angle_delta_uv']} "
                                  f"bflags {bk['flags']:#x}  first px ({x},{y}) fast {pa[y, x]} generic {pb[y, x]}")
                        break
                if len(seen) >= 12:
                    break
    print("identical" if bad == 0 else f"MISMATCH: {bad} pixels")


if __name__ == "__main__":
    main()
