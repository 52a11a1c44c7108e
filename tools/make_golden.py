#!/usr/bin/env python3
"""Generate the committed golden fixtures from the reference decoder (this container only).

For every conformance stream in /root/reference/bits (the reference's own test vectors,
driven by testscript/conformance.py:107-141) this runs oracle/_ref/refdump -- the harness
that decodes with the reference and serialises each frame's av1r batch plus per-stage
MD5s -- and writes

  tests/golden/batches/<stream>.av1b.gz   the frame batches (input to every backend)
  tests/golden/hashes/<stream>.txt        per-frame recon/LF/CDEF/LR MD5s + output MD5

It also copies bits/bits.md5 (expected whole-output MD5s, the conformance pins) to
tests/golden/bits.md5.  Nothing from the reference's sources is copied.

usage: python tools/make_golden.py [--streams a,b,...] [-j N]
"""
import argparse
import concurrent.futures as cf
import gzip
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("AV1DEC_REF", "/root/reference")
REFDUMP = os.path.join(ROOT, "oracle", "_ref", "refdump")
GOLD = os.path.join(ROOT, "tests", "golden")


def one(stream):
    src = os.path.join(REF, "bits", stream + ".ivf")
    with tempfile.TemporaryDirectory() as td:
        b = os.path.join(td, "x.av1b")
        h = os.path.join(td, "x.txt")
        r = subprocess.run([REFDUMP, src, b, h], capture_output=True, text=True)
        if r.returncode != 0:
            return stream, False, r.stderr.strip()[-200:]
        # mtime=0: the same batches give byte-identical fixtures (regeneration is checkable)
        with open(b, "rb") as f, open(os.path.join(GOLD, "batches", stream + ".av1b.gz"), "wb") as raw, \
                gzip.GzipFile(fileobj=raw, mode="wb", compresslevel=9, mtime=0) as g:
            shutil.copyfileobj(f, g)
        shutil.copy(h, os.path.join(GOLD, "hashes", stream + ".txt"))
    return stream, True, ""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="")
    ap.add_argument("-j", type=int, default=6)
    a = ap.parse_args()
    if not os.path.exists(REFDUMP):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "ref"])
    os.makedirs(os.path.join(GOLD, "batches"), exist_ok=True)
    os.makedirs(os.path.join(GOLD, "hashes"), exist_ok=True)
    shutil.copy(os.path.join(REF, "bits", "bits.md5"), os.path.join(GOLD, "bits.md5"))
    streams = a.streams.split(",") if a.streams else sorted(
        f[:-4] for f in os.listdir(os.path.join(REF, "bits")) if f.endswith(".ivf"))
    bad = 0
    with cf.ThreadPoolExecutor(a.j) as ex:
        for s, ok, err in ex.map(one, streams):
            if not ok:
                bad += 1
                print("FAIL", s, err)
    print(f"{len(streams) - bad}/{len(streams)} streams dumped")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
