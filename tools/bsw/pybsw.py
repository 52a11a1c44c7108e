"""Python binding of the synthetic AV1 bitstream writer (tools/bsw/bsw.cpp).

`stream(name)` writes one of the named configurations of CONFIGS as a list of temporal units
(IVF frame payloads); `ivf()` wraps them in an IVF file.  The writer is deterministic: a
configuration always yields the same bytes, which tests/golden/bsw.json pins by SHA-256 next
to the reference decoder's MD5 of the decoded output."""
import ctypes as C
import hashlib
import os
import threading
import struct
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PARSE = os.path.join(ROOT, "av1dec_amd", "csrc", "parse")
BUILD = os.path.join(ROOT, "tools", "_build")
LIB = os.path.join(BUILD, "libav1bsw.so")
CLI = os.path.join(BUILD, "av1bsw")
SRCS = [os.path.join(HERE, "bsw.cpp"), os.path.join(PARSE, "obu.cpp"), os.path.join(PARSE, "block.cpp")]

# name -> writer parameters (+ frames).  S1 / S2 / S3 are SURVEY.md §8(d)'s synthetic
# configurations; the small ones pin features the conformance set never executes (SURVEY
# §8c K6: multi-tile, > CIF sizes, loop-filter sharpness, delta_lf_multi, non-translational
# global motion) against the reference decoder.
BASE = dict(width=1920, height=1080, seed=0x5EED0001, sb128=1, tile_cols_log2=0, tile_rows_log2=0, base_q_idx=96,
            key_interval=0, lf_level=(32, 32, 16, 16), lf_sharpness=0, lf_delta_update=0, delta_q=0, gm=0, cdef=4,
            lr=1, intra_only=0, hidden=0)
CONFIGS = {
    "cif_s1": dict(width=352, height=288, frames=10, seed=0x5EED0101),
    "cif_intra": dict(width=352, height=288, frames=3, seed=0x5EED0102, intra_only=1, base_q_idx=40),
    "cif_sharp_deltalf": dict(width=352, height=288, frames=6, seed=0x5EED0103, lf_sharpness=5, delta_q=3,
                              lf_delta_update=1),
    "cif_deltalf_single": dict(width=352, height=288, frames=4, seed=0x5EED0104, lf_sharpness=2, delta_q=2),
    "cif_gm_translation": dict(width=352, height=288, frames=5, seed=0x5EED0105, gm=1),
    "cif_gm_rotzoom": dict(width=352, height=288, frames=6, seed=0x5EED0106, gm=2),
    "cif_gm_affine_sb64": dict(width=352, height=288, frames=6, seed=0x5EED0107, gm=3, sb128=0),
    "cif_lr_switchable": dict(width=352, height=288, frames=5, seed=0x5EED0108, lr=2, cdef=3, sb128=0),
    "640x360_tiles2x2_sb64": dict(width=640, height=360, frames=5, seed=0x5EED0109, sb128=0, tile_cols_log2=1,
                                  tile_rows_log2=1),
    "odd_416x234_key3": dict(width=416, height=234, frames=7, seed=0x5EED010A, key_interval=3, base_q_idx=180),
    "1080p_s1": dict(width=1920, height=1080, frames=6, seed=0x5EED1000),
    # hidden (show_frame = 0) ALTREF-style frames with future order hints, shown two units
    # later by show_existing_frame units: output order != decode order, backward references
    "cif_hidden": dict(width=352, height=288, frames=12, seed=0x5EED010B, hidden=1),
    "4k_s2_tiles4x2": dict(width=3840, height=2160, frames=3, seed=0x5EED0002, tile_cols_log2=2, tile_rows_log2=1),
}


class Params(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("seed", C.c_uint32), ("sb128", C.c_int),
                ("tile_cols_log2", C.c_int), ("tile_rows_log2", C.c_int), ("base_q_idx", C.c_int),
                ("key_interval", C.c_int), ("lf_level", C.c_int * 4), ("lf_sharpness", C.c_int),
                ("lf_delta_update", C.c_int), ("delta_q", C.c_int), ("gm", C.c_int), ("cdef", C.c_int),
                ("lr", C.c_int), ("verify", C.c_int), ("intra_only", C.c_int), ("hidden", C.c_int)]


def _stale(target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    deps = SRCS + [os.path.join(PARSE, f) for f in os.listdir(PARSE)] + [os.path.join(ROOT, "include", "av1r.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False):
    """libav1bsw.so (ctypes) and the av1bsw command-line writer, in-tree."""
    os.makedirs(BUILD, exist_ok=True)
    common = ["g++", "-std=c++17", "-O2", "-Wall", "-Wno-class-memaccess", "-DAV1P_WRITER",
              "-I" + os.path.join(ROOT, "include"), "-I" + PARSE]
    for target, extra in ((LIB, ["-shared", "-fPIC"]), (CLI, ["-DAV1BSW_MAIN"])):
        if force or _stale(target):
            tmp = f"{target}.{os.getpid()}.{threading.get_ident()}.tmp"
            subprocess.check_call(common + extra + SRCS + ["-o", tmp])
            os.replace(tmp, target)
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
        if _stale(LIB):
            build()
        l = C.CDLL(LIB)
        l.av1bsw_open.restype = C.c_void_p
        l.av1bsw_open.argtypes = [C.POINTER(Params)]
        l.av1bsw_next.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_size_t)]
        l.av1bsw_error.restype = C.c_char_p
        l.av1bsw_error.argtypes = [C.c_void_p]
        l.av1bsw_symbols.restype = C.c_int64
        l.av1bsw_symbols.argtypes = [C.c_void_p]
        l.av1bsw_close.argtypes = [C.c_void_p]
        _lib = l
    return _lib


def params(name=None, **kw):
    d = dict(BASE)
    if name is not None:
        d.update(CONFIGS[name])
    d.update(kw)
    frames = d.pop("frames", 1)
    return d, frames


def write(frames=None, verify=False, name=None, **kw):
    """Temporal units of configuration `name` (overridden by kw), frames 0..frames-1."""
    d, n = params(name, **kw)
    if frames is not None:
        n = frames
    p = Params()
    for k, v in d.items():
        if k == "lf_level":
            p.lf_level[:] = list(v)
        else:
            setattr(p, k, int(v))
    p.verify = int(verify)
    l = lib()
    h = l.av1bsw_open(C.byref(p))
    if not h:
        raise ValueError(f"bad writer parameters {d}")
    out = []
    try:
        for _ in range(n):
            ptr = C.POINTER(C.c_uint8)()
            sz = C.c_size_t()
            if l.av1bsw_next(h, C.byref(ptr), C.byref(sz)) != 0:
                raise RuntimeError("av1bsw: " + l.av1bsw_error(h).decode())
            out.append(C.string_at(ptr, sz.value))
    finally:
        l.av1bsw_close(h)
    return out


def ivf(tus, width, height):
    """An IVF file around the temporal units (the layout tests/DecodeInput.cpp reads)."""
    out = bytearray(b"DKIF" + struct.pack("<HH4sHHIIII", 0, 32, b"AV01", width, height, 30, 1, len(tus), 0))
    for i, tu in enumerate(tus):
        out += struct.pack("<IQ", len(tu), i) + tu
    return bytes(out)


def stream_ivf(name, verify=False, **kw):
    d, _ = params(name, **kw)
    return ivf(write(name=name, verify=verify, **kw), d["width"], d["height"])


def sha256(data):
    return hashlib.sha256(data).hexdigest()
