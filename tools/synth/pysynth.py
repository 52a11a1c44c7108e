"""Python binding of the synthetic frame-batch generator (tools/synth/synth.cpp)."""
import ctypes as C
import os
import threading
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(ROOT, "tools", "_build", "libsynth.so")


def build(force=False):
    src = os.path.join(HERE, "synth.cpp")
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(
            os.path.getmtime(src), os.path.getmtime(os.path.join(ROOT, "include", "av1r.h"))):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        tmp = f"{LIB}.{os.getpid()}.{threading.get_ident()}.tmp"  # build aside, then rename: concurrent test workers never see a partial file
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-shared", "-fPIC", "-I" + os.path.join(ROOT, "include"),
                               src, "-o", tmp])
        os.replace(tmp, LIB)
    return LIB


_lib = None
_lib_lock = threading.Lock()  # threads of one process (bench's IVF writers) build once


def lib():
    global _lib
    with _lib_lock:
        return _lib_locked()


def _lib_locked():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        l = C.CDLL(LIB)
        l.av1r_synth_open.restype = C.c_void_p
        l.av1r_synth_open.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32]
        l.av1r_synth_next.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_size_t)]
        l.av1r_synth_close.argtypes = [C.c_void_p]
        _lib = l
    return _lib


def stream(width, height, nframes, seed, sb128=True, tiles=(1, 1)):
    """Generate `nframes` frames (frame 0 key, then inter) as batchfile.Frame objects."""
    import struct
    from av1dec_amd import batchfile
    l = lib()
    h = l.av1r_synth_open(width, height, int(sb128), tiles[0], tiles[1], seed)
    if not h:
        raise ValueError("bad synth parameters")
    out = []
    try:
        for _ in range(nframes):
            p = C.POINTER(C.c_uint8)()
            n = C.c_size_t()
            if l.av1r_synth_next(h, C.byref(p), C.byref(n)) != 0:
                raise RuntimeError("synth failed")
            rec = bytes(np.ctypeslib.as_array(p, shape=(n.value,)))
            out.extend(batchfile.parse(b"AV1B" + struct.pack("<I", batchfile.abi.AV1R_VERSION) + rec))
    finally:
        l.av1r_synth_close(h)
    return out
