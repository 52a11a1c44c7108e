#!/usr/bin/env python3
"""CPU-baseline calibration at the bench's resolution: k_1080p =
reference fps / oracle fps on the SAME 1080p frames -- the writer's 1080p_s1 stream
(tools/bsw: 1 key + inter frames, the bench's synthetic distributions) -- on the same CPU
(this container), 1 thread each.  The reference is oracle/_ref/av1dec_ref (the reference CLI,
-O1); its "decode fps" includes its own parse, so k_1080p converts the oracle's
reconstruction-only rate into a parse-inclusive reference-equivalent rate.  The inter frames
dominate this stream as they dominate the bench's GOP.  Adds "k_1080p" to
profiles/cpu_calibration.json.  usage: python tools/calibrate_k_1080p.py [frames]"""
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools", "bsw")]
import pybsw  # noqa: E402
import pyoracle  # noqa: E402
from av1dec_amd import parser  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "av1dec_ref")
OUT = os.path.join(ROOT, "profiles", "cpu_calibration.json")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    data = pybsw.stream_ivf("1080p_s1", frames=n, seed=0x5EED1000)
    with tempfile.NamedTemporaryFile(suffix=".ivf") as f:
        f.write(data)
        f.flush()
        out = subprocess.run([REF, "-i", f.name], capture_output=True, text=True, timeout=3600).stdout
    ref = float(re.findall(r"decode fps = ([0-9.]+)", out)[-1])
    frames = parser.Parser().decode_ivf(data)
    best = None
    for _ in range(2):
        o = pyoracle.Oracle(keep_stages=False)
        t = time.perf_counter()
        for fr in frames:
            o.decode_frame(fr)
            while o.output_pending():
                o.get_output()
        dt = time.perf_counter() - t
        o.close()
        best = dt if best is None else min(best, dt)
    orc = len(frames) / best
    cal = json.load(open(OUT))
    cal["k_1080p"] = {"k": round(ref / orc, 4), "reference_fps": round(ref, 4), "oracle_fps": round(orc, 4),
                      "frames": n, "stream": f"tools/bsw 1080p_s1 seed 0x5eed1000, {n} frames (1 key + {n - 1} inter)",
                      "cpu_model": cal.get("cpu_model"),
                      "note": "same frames, same CPU, 1 thread; reference 'decode fps' includes its parse, the "
                              "oracle's reconstruction + filters from the parsed batches do not"}
    json.dump(cal, open(OUT, "w"), indent=1)
    print(json.dumps(cal["k_1080p"]))


if __name__ == "__main__":
    main()
