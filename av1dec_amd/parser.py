"""Host AV1 parser (include/av1p.h): IVF/OBU bytes -> av1r frame batches.

The parse half of the reference decoder (oddstone/av1dec: Decoder::decode,
decoder/Av1Decoder.cpp:49-109, and the Parser / Tile / Block / TransformBlock syntax) as a
native library, libav1p.so.  `Parser.decode_tu()` returns the frame batches a temporal unit
completes, as `batchfile.Frame` objects (numpy copies of the native arrays), ready for
`Decoder.decode_frame`, `Decoder.pack` or the oracle."""
import ctypes as C
import struct

import numpy as np

from . import abi, batchfile, native


def ivf_frames(data):
    """Yield the payload of every frame of an IVF file (tests/IvfReader: 32-byte file header,
    then a 12-byte header -- u32 size, u64 timestamp -- per frame)."""
    if data[:4] != b"DKIF":
        raise ValueError("not an IVF file")
    hdr_len = struct.unpack_from("<H", data, 6)[0] or 32
    pos = hdr_len
    while pos + 12 <= len(data):
        sz = struct.unpack_from("<I", data, pos)[0]
        pos += 12
        if pos + sz > len(data):
            break
        yield data[pos:pos + sz]
        pos += sz


def _copy(ptr, nbytes):
    if not nbytes:
        return np.zeros(0, dtype=np.uint8)
    return np.frombuffer(C.string_at(ptr, nbytes), dtype=np.uint8).copy()


def frame_from_batch(ptr):
    """Copy a native av1r_frame_batch (pointer) into a batchfile.Frame."""
    b = abi.FrameBatch.from_address(ptr)
    hdr = abi.FrameHdr.from_address(b.hdr)
    secs = {"hdr": _copy(b.hdr, C.sizeof(abi.FrameHdr))}
    n_mi = 0 if hdr.show_existing_frame or not b.mi else hdr.mi_rows_alloc * hdr.mi_stride
    secs["mi"] = _copy(b.mi, n_mi * abi.SIZEOF_MI)
    secs["blocks"] = _copy(b.blocks, b.n_blocks * abi.SIZEOF_BLOCK)
    secs["tbs"] = _copy(b.tbs, b.n_tbs * abi.SIZEOF_TB)
    secs["coefs"] = _copy(b.coefs, b.n_coefs * 4)
    secs["palette"] = _copy(b.palette, b.n_palette)
    n_cdef = 0 if hdr.show_existing_frame else hdr.cdef_rows * hdr.cdef_cols
    secs["cdef"] = _copy(b.cdef_idx, n_cdef)
    secs["lr"] = _copy(b.lr_units, b.n_lr_units * abi.SIZEOF_LR_UNIT)
    return batchfile.Frame(secs)


class ParseError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"av1p status {status}: {msg}")
        self.status = status


class Parser:
    """One parsing context (one stream).  Not thread-safe; use one per thread."""

    def __init__(self, tile_threads=None, mode_info=True):
        self._l = native.parser_lib()
        h = C.c_void_p()
        rc = self._l.av1p_create(C.byref(h))
        if rc:
            raise ParseError(rc, "av1p_create failed")
        self._h = h
        if tile_threads is not None:
            rc = self._l.av1p_set_tile_threads(h, int(tile_threads))
            if rc:
                raise ParseError(rc, f"av1p_set_tile_threads({tile_threads})")
        if not mode_info:  # frames carry no mode-info grid (av1p_set_mode_info)
            self._l.av1p_set_mode_info(h, 0)

    def decode_tu(self, data):
        n = C.c_int(0)
        rc = self._l.av1p_decode_tu(self._h, bytes(data), len(data), C.byref(n))
        if rc:
            raise ParseError(rc, self._l.av1p_last_error(self._h).decode())
        return [frame_from_batch(self._l.av1p_frame(self._h, i)) for i in range(n.value)]

    def decode_ivf(self, data):
        """All frame batches of an IVF stream, in decode order."""
        out = []
        for tu in ivf_frames(data):
            out += self.decode_tu(tu)
        return out

    def close(self):
        if self._h:
            self._l.av1p_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
