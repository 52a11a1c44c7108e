#!/usr/bin/env python3
"""Device time of one synthetic 1080p key frame alone on the chip, k_flow against k_strip
(av1r_set_strip_levels), and a check that both reconstruct it identically.
usage (GPU box): python3 tools/keyframe_time.py [reps] [k_flow|k_strip]  (one kernel only: PMC passes)"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    import pysynth
    from av1dec_amd import Decoder, native
    L = native.lib()
    frames = pysynth.stream(1920, 1080, 2, 0x5EED1000, sb128=True)
    out = {}
    only = sys.argv[2] if len(sys.argv) > 2 else None
    for name, lv in (("k_flow", 0), ("k_strip", 400)):
        if only and name != only:
            continue
        L.av1r_set_strip_levels(lv)
        d = Decoder(0, keep_stages=True, timing=True)
        h = d.prepare(frames[0])
        times = []
        for _ in range(reps):
            d.decode_prepared(h)
            d.synchronize()
            times.append(d.last_frame_times())
        d.decode_frame(frames[0])
        m = hashlib.md5()
        for p in d.read_stage(0):
            m.update(p.tobytes())
        recon = sorted(t[0] for t in times)
        out[name] = m.hexdigest()
        print(f"{name:8s} key frame recon ms: min {recon[0]:.3f} median {recon[len(recon) // 2]:.3f} "
              f"max {recon[-1]:.3f}  (LF {times[-1][1]:.3f} CDEF {times[-1][2]:.3f} LR {times[-1][3]:.3f})  md5 {out[name]}")
        d.release_prepared(h)
        d.close()
    L.av1r_set_strip_levels(400)
    print("identical" if len(set(out.values())) == 1 else "MISMATCH")


if __name__ == "__main__":
    main()
