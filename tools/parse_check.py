#!/usr/bin/env python3
"""Compare the host parser's frame batches with the tree-walker fixtures
(tests/golden/batches/<stream>.av1b.gz, written by oracle/harness/refdump from the
reference decoder's parse trees), frame by frame and field by field.

    python tools/parse_check.py [stream ...]      (default: every stream with a fixture)
"""
import gzip
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from av1dec_amd import abi, batchfile, native  # noqa: E402
from av1dec_amd.parser import Parser  # noqa: E402
import golden  # noqa: E402

# header fields a show_existing_frame record carries (the rest is not read for it)
SHOW_EXISTING_FIELDS = ("show_existing_frame", "frame_to_show", "refresh_frame_flags", "frame_type")


def hdr_diff(a, b):
    out = []
    if a.show_existing_frame or b.show_existing_frame:
        names = SHOW_EXISTING_FIELDS
    else:
        names = [f[0] for f in abi.FrameHdr._fields_ if f[0] != "reserved"]
    for n in names:
        x, y = getattr(a, n), getattr(b, n)
        if hasattr(x, "__len__"):
            x, y = np.ctypeslib.as_array(x).tolist(), np.ctypeslib.as_array(y).tolist()
            if n.startswith("cdef_") and n[5:] in ("y_pri", "y_sec", "uv_pri", "uv_sec"):
                k = 1 << a.cdef_bits  # strengths past 1 << cdef_bits are never read
                x, y = x[:k], y[:k]
        if x != y:
            out.append(f"hdr.{n}: parser {x} fixture {y}")
    return out


def rec_diff(name, a, b, dtype, limit=3):
    if a.size != b.size:
        return [f"{name}: {a.size} vs {b.size} bytes"]
    if np.array_equal(a, b):
        return []
    ra, rb = a.view(dtype), b.view(dtype)
    bad = np.nonzero(ra != rb)[0]
    out = [f"{name}: {len(bad)} records differ"]
    for i in bad[:limit]:
        fields = [f for f in dtype.names if not np.array_equal(ra[i][f], rb[i][f])]
        out.append(f"  [{i}] " + ", ".join(f"{f}: {ra[i][f].tolist()} vs {rb[i][f].tolist()}" for f in fields))
    return out


def compare(frames, gold):
    problems = []
    if len(frames) != len(gold):
        problems.append(f"frame count {len(frames)} vs {len(gold)}")
    for k, (f, g) in enumerate(zip(frames, gold)):
        d = hdr_diff(f.hdr, g.hdr)
        if not f.show_existing:
            d += rec_diff("mi", f.sec["mi"], g.sec["mi"], abi.MI_DTYPE)
            d += rec_diff("blocks", f.sec["blocks"], g.sec["blocks"], abi.BLOCK_DTYPE)
            d += rec_diff("tbs", f.sec["tbs"], g.sec["tbs"], abi.TB_DTYPE)
            for s in ("coefs", "palette", "cdef", "lr"):
                if not np.array_equal(f.sec[s], g.sec[s]):
                    d.append(f"{s}: differs ({f.sec[s].size} vs {g.sec[s].size} bytes)")
        if d:
            problems.append(f"frame {k}:")
            problems += ["  " + x for x in d[:12]]
            break
    return problems


def main():
    native.build_parser()
    streams = sys.argv[1:] or golden.streams()
    ok = 0
    for s in streams:
        data = open(golden.ivf_path(s), "rb").read()
        try:
            frames = Parser().decode_ivf(data)
        except Exception as e:  # noqa: BLE001
            print(f"{s}: EXCEPTION {e}")
            continue
        probs = compare(frames, batchfile.load(golden.batch_path(s)))
        if probs:
            print(f"{s}: MISMATCH")
            for p in probs:
                print("   ", p)
        else:
            ok += 1
            print(f"{s}: ok ({len(frames)} frames)")
    print(f"{ok}/{len(streams)} streams identical")


if __name__ == "__main__":
    main()
