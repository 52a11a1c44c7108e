"""Reader/writer for .av1b frame-batch streams (the host->device boundary payload).

File layout (little-endian): b"AV1B", u32 version, then per frame b"FRME", u32 length,
and eight sections (u32 byte length + bytes, padded to 4): frame header, mi grid,
blocks, transform blocks, coefficients, palette blob, cdef_idx, lr units -- the arrays
of av1r_frame_batch (include/av1r.h).  Files may be gzip-compressed (.gz)."""
import ctypes as C
import gzip
import struct

import numpy as np

from . import abi

SECTIONS = ("hdr", "mi", "blocks", "tbs", "coefs", "palette", "cdef", "lr")


class Frame:
    """One frame's batch; keeps the backing buffers alive while `batch` is used."""

    def __init__(self, sections):
        self.sec = sections
        self.hdr = abi.FrameHdr.from_buffer_copy(sections["hdr"].tobytes())
        self._keep = {}
        b = abi.FrameBatch()
        hb = np.frombuffer(sections["hdr"].tobytes(), dtype=np.uint8).copy()
        self._keep["hdr"] = hb
        b.hdr = hb.ctypes.data
        for name, field in (("mi", "mi"), ("blocks", "blocks"), ("tbs", "tbs"), ("coefs", "coefs"),
                            ("palette", "palette"), ("cdef", "cdef_idx"), ("lr", "lr_units")):
            arr = sections[name]
            if arr.size == 0:
                arr = np.zeros(4, dtype=np.uint8)
            arr = np.ascontiguousarray(arr)
            self._keep[name] = arr
            setattr(b, field, arr.ctypes.data)
        b.n_blocks = sections["blocks"].size // abi.SIZEOF_BLOCK
        b.n_tbs = sections["tbs"].size // abi.SIZEOF_TB
        b.n_coefs = sections["coefs"].size // 4
        b.n_palette = sections["palette"].size
        b.n_lr_units = sections["lr"].size // abi.SIZEOF_LR_UNIT
        self.batch = b

    @property
    def show_existing(self):
        return bool(self.hdr.show_existing_frame)

    @property
    def n_blocks(self):
        return self.batch.n_blocks

    @property
    def n_tbs(self):
        return self.batch.n_tbs

    def byref(self):
        return C.byref(self.batch)

    def payload_bytes(self):
        return sum(int(a.size) for a in self.sec.values())

    def to_bytes(self):
        out = bytearray()
        for name in SECTIONS:
            a = self.sec[name].tobytes()
            out += struct.pack("<I", len(a)) + a
            while len(out) & 3:
                out += b"\0"
        return b"FRME" + struct.pack("<I", len(out)) + bytes(out)


def parse(data):
    if data[:4] != b"AV1B":
        raise ValueError("not an av1b stream")
    ver = struct.unpack_from("<I", data, 4)[0]
    if ver != abi.AV1R_VERSION:
        raise ValueError(f"av1b version {ver} != {abi.AV1R_VERSION}")
    pos = 8
    frames = []
    buf = np.frombuffer(data, dtype=np.uint8)
    while pos + 8 <= len(data):
        magic = data[pos:pos + 4]
        n = struct.unpack_from("<I", data, pos + 4)[0]
        if magic != b"FRME":
            raise ValueError("bad frame record")
        p = pos + 8
        end = p + n
        secs = {}
        for name in SECTIONS:
            ln = struct.unpack_from("<I", data, p)[0]
            p += 4
            secs[name] = buf[p:p + ln]
            p += (ln + 3) & ~3
        if p != end:
            raise ValueError("frame record length mismatch")
        frames.append(Frame(secs))
        pos = end
    return frames


def load(path):
    opener = gzip.open if str(path).endswith(".gz") else open
    with opener(path, "rb") as f:
        return parse(f.read())


def write(path, frames):
    opener = gzip.open if str(path).endswith(".gz") else open
    with opener(path, "wb") as f:
        f.write(b"AV1B" + struct.pack("<I", abi.AV1R_VERSION))
        for fr in frames:
            f.write(fr.to_bytes())
