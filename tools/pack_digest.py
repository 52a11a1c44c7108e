#!/usr/bin/env python3
"""MD5 over the packed bytes (av1r_pack, host only) of the committed fixture streams and a
few synthetic 1080p frames: the packed batch is a pure function of the frame, so two
packing code paths (e.g. AV1R_PACK_FUSED=0/1) must print the same digest.
usage: python3 tools/pack_digest.py [max_streams]"""
import ctypes as C
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))
from av1dec_amd import native, batchfile
import golden, bench
l = native.lib()
def packed(fr):
    p = C.c_void_p()
    rc = l.av1r_pack(C.cast(fr.byref(), C.c_void_p), C.byref(p))
    if rc: return 'ERR%d' % rc
    n = C.c_size_t()
    ptr = l.av1r_packed_data(p, C.byref(n))
    h = hashlib.md5(C.string_at(ptr, n.value)).hexdigest()
    l.av1r_packed_free(p)
    return h
frames = []
for s in golden.streams()[:int(sys.argv[1]) if len(sys.argv) > 1 else None]:
    frames += batchfile.load(golden.batch_path(s))
frames += bench.rank_streams("1080p", 0, 1, 6)[0]
out = [packed(f) for f in frames if not f.show_existing]
if os.environ.get("PD_VERBOSE"): print("\n".join(out), file=sys.stderr)
print(hashlib.md5("".join(out).encode()).hexdigest(), len(out))
