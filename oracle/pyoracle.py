"""Python binding of the CPU oracle (oracle/av1r_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the av1dec_amd product package."""
import ctypes as C
import hashlib
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "oracle"])


def _load():
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    lib.oracle_create.restype = C.c_void_p
    lib.oracle_destroy.argtypes = [C.c_void_p]
    lib.oracle_decode_frame.argtypes = [C.c_void_p, C.c_void_p]
    lib.oracle_show_existing.argtypes = [C.c_void_p, C.c_int, C.c_int]
    lib.oracle_output_pending.argtypes = [C.c_void_p]
    lib.oracle_get_output.argtypes = [C.c_void_p] + [C.c_void_p, C.c_int] * 3 + [C.c_void_p, C.c_void_p]
    lib.oracle_read_stage.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int]
    lib.oracle_set_keep_stages.argtypes = [C.c_void_p, C.c_int]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


class Oracle:
    """Same surface as av1dec_amd.Decoder, computed serially on the CPU."""

    def __init__(self, keep_stages=True):
        self.l = lib()
        self.c = self.l.oracle_create()
        self.l.oracle_set_keep_stages(self.c, int(keep_stages))
        self.last = None

    def close(self):
        if self.c:
            self.l.oracle_destroy(self.c)
            self.c = None

    __del__ = close

    def decode_frame(self, frame):
        self.last = frame.hdr
        rc = self.l.oracle_decode_frame(self.c, C.cast(frame.byref(), C.c_void_p))
        if rc != 0:
            raise RuntimeError(f"oracle_decode_frame failed: {rc}")

    def output_pending(self):
        return self.l.oracle_output_pending(self.c)

    def get_output(self):
        w = C.c_int()
        h = C.c_int()
        if self.l.oracle_get_output(self.c, None, 0, None, 0, None, 0, C.byref(w), C.byref(h)) != 0:
            return None
        W, H = w.value, h.value
        y = np.empty((H, W), np.uint8)
        u = np.empty((H >> 1, W >> 1), np.uint8)
        v = np.empty((H >> 1, W >> 1), np.uint8)
        self.l.oracle_get_output(self.c, y.ctypes.data, W, u.ctypes.data, W >> 1, v.ctypes.data, W >> 1, None, None)
        return y, u, v

    def read_stage(self, stage):
        W, H = self.last.frame_width, self.last.frame_height
        planes = []
        for p in range(3):
            w, h = (W, H) if p == 0 else (W >> 1, H >> 1)
            a = np.empty((h, w), np.uint8)
            if self.l.oracle_read_stage(self.c, stage, p, a.ctypes.data, w) != 0:
                raise RuntimeError("no stage")
            planes.append(a)
        return planes


def md5_planes(planes):
    m = hashlib.md5()
    for p in planes:
        m.update(np.ascontiguousarray(p).tobytes())
    return m.hexdigest()
