"""CPU-baseline calibration: k = reference fps / oracle fps on the same
conformance streams, measured in THIS container (the reference cannot travel to the GPU
box).  The reference is oracle/_ref/av1dec_ref, the reference CLI built -O1 from its own
sources (oracle/Makefile); its "decode fps" (tests/Av1Dec.cpp:83-92) times
Decoder::decode, which includes the reference's parse.  The oracle (oracle/av1r_oracle.c)
decodes the same frames from their batches (no parse).  Both single-threaded, median of 3.
bench.py scales the oracle's fps measured on the GPU box's host by k to report a
reference-equivalent fps.  Writes profiles/cpu_calibration.json.
usage: python tools/calibrate_k.py"""
import json
import os
import platform
import re
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import golden  # noqa: E402
import pyoracle  # noqa: E402
from av1dec_amd import batchfile  # noqa: E402

STREAMS = ["av1-1-b8-02-allintra", "av1-1-b8-06-mfmv", "av1-1-b8-04-cdfupdate", "av1-1-b8-00-quantizer-20",
           "av1-1-b8-00-quantizer-40", "av1-1-b8-01-size-66x66", "av1-1-b8-03-sizeup"]
REF = os.path.join(ROOT, "oracle", "_ref", "av1dec_ref")
BITS = os.environ.get("AV1DEC_BITS", "/root/reference/bits")


def ref_fps(path):
    out = subprocess.run([REF, "-i", path], capture_output=True, text=True, timeout=600).stdout
    m = re.findall(r"decode fps = ([0-9.]+)", out)
    return float(m[-1])


def oracle_time(frames):
    o = pyoracle.Oracle(keep_stages=False)
    t = time.perf_counter()
    for f in frames:
        o.decode_frame(f)
        while o.output_pending():
            o.get_output()
    dt = time.perf_counter() - t
    o.close()
    return dt


def main():
    rows = []
    for s in STREAMS:
        ivf = os.path.join(BITS, s + ".ivf")
        if not os.path.exists(ivf) or not os.path.exists(golden.batch_path(s)):
            continue
        frames = batchfile.load(golden.batch_path(s))
        n = sum(1 for f in frames if not f.show_existing)
        r = statistics.median(ref_fps(ivf) for _ in range(3))
        o = n / statistics.median(oracle_time(frames) for _ in range(3))
        rows.append({"stream": s, "frames": n, "reference_fps": round(r, 3), "oracle_fps": round(o, 3),
                     "k": round(r / o, 4)})
        print(rows[-1], flush=True)
    tot = sum(x["frames"] for x in rows)
    ref_t = sum(x["frames"] / x["reference_fps"] for x in rows)
    ora_t = sum(x["frames"] / x["oracle_fps"] for x in rows)
    model = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")), platform.processor())
    res = {"k": round(ora_t / ref_t, 4), "reference_fps": round(tot / ref_t, 3), "oracle_fps": round(tot / ora_t, 3),
           "frames": tot, "streams": rows, "cpu_model": model, "host_cores": os.cpu_count(),
           "reference_build": "oracle/_ref/av1dec_ref: the reference CLI, -O1 (fastest bit-exact build), its "
                              "'decode fps' (Decoder::decode incl. the reference's parse)",
           "oracle_build": "oracle/av1r_oracle.c -O2 via ctypes, from batches (no parse)",
           "note": "k = reference fps / oracle fps on the same frames, 1 thread each, median of 3"}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "streams"}))


if __name__ == "__main__":
    main()
