"""Host parser (include/av1p.h, libav1p.so) against the reference's parse trees.

The fixtures tests/golden/batches/*.av1b.gz are the reference decoder's own parse of each
conformance stream, serialised by oracle/harness/refdump; the parser must reproduce every
byte of every frame batch from the bitstream alone.  The bitstreams are read from the
reference checkout (not part of this repository), so these tests run in the build
container and skip elsewhere.  CPU only: the parser is host code."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import golden  # noqa: E402
from av1dec_amd import abi, batchfile, native  # noqa: E402

needs_bits = pytest.mark.skipif(not golden.have_ivf(), reason="conformance bitstreams (reference checkout) absent")


@pytest.fixture(scope="module")
def parser_mod():
    native.build_parser()
    from av1dec_amd import parser
    return parser


def _frames(parser_mod, stream):
    with open(golden.ivf_path(stream), "rb") as f:
        return parser_mod.Parser().decode_ivf(f.read())


SHOW_EXISTING_FIELDS = ("show_existing_frame", "frame_to_show", "refresh_frame_flags", "frame_type")


def _same(f, g):
    if f.show_existing or g.show_existing:
        return all(getattr(f.hdr, n) == getattr(g.hdr, n) for n in SHOW_EXISTING_FIELDS)
    return all(np.array_equal(f.sec[s], g.sec[s]) for s in batchfile.SECTIONS)


@needs_bits
@pytest.mark.parametrize("stream", golden.streams())
def test_parser_matches_reference_parse(parser_mod, stream):
    frames = _frames(parser_mod, stream)
    gold = batchfile.load(golden.batch_path(stream))
    assert len(frames) == len(gold)
    for k, (f, g) in enumerate(zip(frames, gold)):
        assert _same(f, g), f"{stream}: frame {k} differs from the reference's parse"


def test_parser_exports_and_structs():
    native.build_parser()
    lib = native.parser_lib()
    for name in native.PARSE_EXPORTS:
        assert hasattr(lib, name)


@needs_bits
def test_parser_rejects_damage_without_crashing(parser_mod):
    with open(golden.ivf_path("av1-1-b8-01-size-16x16"), "rb") as f:
        tus = list(parser_mod.ivf_frames(f.read()))
    # truncated temporal units, and random bytes: a status, never a crash
    p = parser_mod.Parser()
    with pytest.raises(parser_mod.ParseError):
        p.decode_tu(tus[0][: len(tus[0]) // 3])
    rng = np.random.default_rng(7)
    for _ in range(20):
        p = parser_mod.Parser()
        try:
            p.decode_tu(rng.integers(0, 256, 200, dtype=np.uint8).tobytes())
        except parser_mod.ParseError:
            pass
    # tile data corrupted after a valid header: parse completes or fails cleanly
    bad = bytearray(tus[0])
    for i in range(len(bad) // 2, len(bad)):
        bad[i] ^= 0x5A
    p = parser_mod.Parser()
    try:
        p.decode_tu(bytes(bad))
    except parser_mod.ParseError:
        pass


def test_parser_empty_and_delimiter_only(parser_mod):
    p = parser_mod.Parser()
    assert p.decode_tu(b"") == []
    assert p.decode_tu(bytes([0x12, 0x00])) == []  # temporal delimiter OBU
    with pytest.raises(parser_mod.ParseError):  # a frame header before any sequence header
        p.decode_tu(bytes([0x1A, 0x01, 0x00]))


@needs_bits
def test_parser_streams_are_independent(parser_mod):
    """Two contexts interleaved give the same batches as each alone (no shared state)."""
    a, b = "av1-1-b8-06-mfmv", "av1-1-b8-04-cdfupdate"
    with open(golden.ivf_path(a), "rb") as f:
        ta = list(parser_mod.ivf_frames(f.read()))
    with open(golden.ivf_path(b), "rb") as f:
        tb = list(parser_mod.ivf_frames(f.read()))
    pa, pb = parser_mod.Parser(), parser_mod.Parser()
    fa, fb = [], []
    for i in range(max(len(ta), len(tb))):
        if i < len(ta):
            fa += pa.decode_tu(ta[i])
        if i < len(tb):
            fb += pb.decode_tu(tb[i])
    for stream, frames in ((a, fa), (b, fb)):
        gold = batchfile.load(golden.batch_path(stream))
        assert len(frames) == len(gold)
        assert all(_same(f, g) for f, g in zip(frames, gold))


@needs_bits
@pytest.mark.parametrize("stream", ["av1-1-b8-01-size-16x18", "av1-1-b8-04-cdfupdate", "av1-1-b8-06-mfmv",
                                    "Halo_426x240_1frames_intrabc"])
def test_bitstream_to_pixels_matches_conformance_md5(parser_mod, stream):
    """Bitstream -> host parser -> CPU oracle restatement -> the conformance MD5 (bits.md5):
    the whole decode with nothing from the reference in the loop."""
    import hashlib
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    expect = golden.bits_md5()[stream]
    o = pyoracle.Oracle(keep_stages=False)
    h = hashlib.md5()
    for fr in _frames(parser_mod, stream):
        o.decode_frame(fr)
        while o.output_pending():
            for plane in o.get_output():
                h.update(plane.tobytes())
    o.close()
    assert h.hexdigest() == expect


@pytest.mark.parametrize("name", ["4k_s2_tiles4x2", "640x360_tiles2x2_sb64"])
def test_tile_parallel_parse_is_identical(parser_mod, name):
    """Tiles parsed concurrently (one TileCtx per tile, merged in tile order) give the same
    batches, byte for byte, as the serial parse (Parser::parseTileGroup's tile loop,
    Parser.cpp:492-521)."""
    sys.path.insert(0, os.path.join(ROOT, "tools", "bsw"))
    import pybsw
    data = pybsw.stream_ivf(name, frames=3 if name.startswith("4k") else None)
    serial = parser_mod.Parser(tile_threads=1).decode_ivf(data)
    for n in (2, 8):
        par = parser_mod.Parser(tile_threads=n).decode_ivf(data)
        assert len(par) == len(serial)
        for k, (f, g) in enumerate(zip(par, serial)):
            assert _same(f, g), f"{name}: frame {k} differs with {n} tile threads"


@needs_bits
@pytest.mark.parametrize("name", ["av1-1-b8-01-size-66x66", "av1-1-b8-06-mfmv"])
def test_parse_without_mode_info_grid(parser_mod, name):
    """av1p_set_mode_info(ctx, 0): every section but the mode-info grid is unchanged, and
    that one is empty (the product paths rebuild it on the device)."""
    with open(golden.ivf_path(name), "rb") as f:
        data = f.read()
    full = parser_mod.Parser().decode_ivf(data)
    lean = parser_mod.Parser(mode_info=False).decode_ivf(data)
    assert len(full) == len(lean)
    for f, g in zip(full, lean):
        assert g.sec["mi"].size == 0
        for s in batchfile.SECTIONS:
            if s != "mi":
                assert np.array_equal(f.sec[s], g.sec[s]), s


@needs_bits
def test_two_frame_generations_keep_the_previous_unit(parser_mod):
    """av1p_set_frame_generations(ctx, 2): a unit's frame batches stay intact while the next
    unit is parsed (the native IVF source packs unit g while unit g + 1 parses)."""
    import ctypes as C
    with open(golden.ivf_path("av1-1-b8-01-size-66x66"), "rb") as f:
        tus = list(parser_mod.ivf_frames(f.read()))
    l = native.parser_lib()
    h = C.c_void_p()
    assert l.av1p_create(C.byref(h)) == 0
    try:
        assert l.av1p_set_frame_generations(h, 2) == 0
        assert l.av1p_set_frame_generations(h, 3) != 0
        n = C.c_int()
        prev = None
        for tu in tus:
            assert l.av1p_decode_tu(h, tu, len(tu), C.byref(n)) == 0
            if prev is not None:  # the previous unit's frames, after this unit's parse
                for ptr, frame in prev:
                    again = parser_mod.frame_from_batch(ptr)
                    assert all(np.array_equal(frame.sec[s], again.sec[s]) for s in batchfile.SECTIONS)
            prev = [(p, parser_mod.frame_from_batch(p)) for p in (l.av1p_frame(h, i) for i in range(n.value))]
    finally:
        l.av1p_destroy(h)
