"""The C-ABI library builds for gfx950, loads, exports every entry point of
include/av1r.h, and its struct layouts match the Python mirror and the fixtures."""
import ctypes as C
import os
import re

import golden
from av1dec_amd import abi, batchfile, native


def declared_functions():
    src = open(os.path.join(native.ROOT, "include", "av1r.h")).read()
    return sorted(set(re.findall(r"\b(av1r_\w+)\s*\(", src)) - {"av1r_ctx"})


def test_exports_every_declared_symbol(native_lib):
    decl = declared_functions()
    assert decl, "no declarations parsed"
    for name in decl:
        assert hasattr(native_lib, name), name
    assert sorted(native.EXPORTS) == decl


def test_struct_sizes(native_lib):
    assert native_lib.av1r_sizeof(0) == C.sizeof(abi.FrameHdr)
    assert native_lib.av1r_sizeof(1) == abi.SIZEOF_MI
    assert native_lib.av1r_sizeof(2) == abi.SIZEOF_BLOCK
    assert native_lib.av1r_sizeof(3) == abi.SIZEOF_TB
    assert native_lib.av1r_sizeof(4) == abi.SIZEOF_LR_UNIT
    assert native_lib.av1r_sizeof(5) == C.sizeof(abi.FrameBatch)


def test_batchfile_roundtrip(tmp_path):
    frames = batchfile.load(golden.batch_path("av1-1-b8-06-mfmv"))
    p = tmp_path / "x.av1b.gz"
    batchfile.write(p, frames)
    again = batchfile.load(p)
    assert len(again) == len(frames)
    for a, b in zip(frames, again):
        assert a.to_bytes() == b.to_bytes()
        assert a.hdr.frame_width == 352 and a.n_tbs == b.n_tbs


def test_fixture_records_are_whole(native_lib):
    for s in ("64x64", "av1-1-b8-02-allintra", "Halo_426x240_1frames_intrabc"):
        for fr in batchfile.load(golden.batch_path(s)):
            assert fr.sec["blocks"].size % abi.SIZEOF_BLOCK == 0
            assert fr.sec["tbs"].size % abi.SIZEOF_TB == 0
            assert fr.sec["mi"].size == abi.SIZEOF_MI * fr.hdr.mi_stride * fr.hdr.mi_rows_alloc or fr.show_existing


def test_host_validation_and_schedule_on_all_fixtures(native_lib):
    """Every committed batch passes the backend's host-side validation (the checks that
    guard every index a kernel follows) and yields a dependency schedule."""
    import ctypes as C
    err = C.create_string_buffer(256)
    for s in golden.streams():
        for i, fr in enumerate(batchfile.load(golden.batch_path(s))):
            lv = C.c_int()
            rc = native_lib.av1r_check_batch(C.cast(fr.byref(), C.c_void_p), C.byref(lv), err, 256)
            assert rc == 0, f"{s} frame {i}: {err.value.decode()}"
            if not fr.show_existing:
                assert lv.value >= 1


def test_validation_rejects_bad_batches(native_lib):
    import ctypes as C
    import numpy as np
    fr = batchfile.load(golden.batch_path("av1-1-b8-06-mfmv"))[1]
    err = C.create_string_buffer(256)
    tb = np.frombuffer(fr.sec["tbs"].tobytes(), abi.TB_DTYPE).copy()
    tb["block"][3] = 10 ** 6
    secs = dict(fr.sec)
    secs["tbs"] = tb.view(np.uint8).ravel()
    bad = batchfile.Frame(secs)
    assert native_lib.av1r_check_batch(C.cast(bad.byref(), C.c_void_p), None, err, 256) == abi.AV1R_E_INVALID
    hdr = abi.FrameHdr.from_buffer_copy(fr.sec["hdr"].tobytes())
    hdr.bitdepth = 10
    secs = dict(fr.sec)
    secs["hdr"] = np.frombuffer(bytes(hdr), np.uint8).copy()
    bad = batchfile.Frame(secs)
    assert native_lib.av1r_check_batch(C.cast(bad.byref(), C.c_void_p), None, err, 256) == abi.AV1R_E_UNSUPPORTED
    assert b"8-bit" in err.value


def test_pack_is_host_only_and_thread_safe(native_lib):
    """av1r_pack (validation + flow-only schedule + packing, no context, no device) on
    every frame of several fixture streams from concurrent threads: every frame packs, the
    packed size is stable across threads, and a malformed batch fails with its message."""
    import ctypes as C
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    from av1dec_amd import Decoder
    frames = []
    for s in ("av1-1-b8-06-mfmv", "av1-1-b8-04-cdfupdate", "Halo_426x240_1frames_intrabc", "64x64"):
        frames += batchfile.load(golden.batch_path(s))

    def size(fr):
        p = Decoder.pack(fr)
        n = native_lib.av1r_packed_bytes(p)
        Decoder.free_packed(p)
        return n
    serial = [size(f) for f in frames]
    with ThreadPoolExecutor(4) as ex:
        assert list(ex.map(size, frames * 2)) == serial * 2
    assert all(n > 0 for f, n in zip(frames, serial) if not f.show_existing)
    fr = batchfile.load(golden.batch_path("av1-1-b8-06-mfmv"))[1]
    tb = np.frombuffer(fr.sec["tbs"].tobytes(), abi.TB_DTYPE).copy()
    tb["tx_size"][0] = 99
    secs = dict(fr.sec)
    secs["tbs"] = tb.view(np.uint8).ravel()
    p = C.c_void_p()
    assert native_lib.av1r_pack(C.cast(batchfile.Frame(secs).byref(), C.c_void_p), C.byref(p)) == abi.AV1R_E_INVALID
    assert b"tb 0" in native_lib.av1r_pack_last_error()


def _declared(header, prefix):
    src = open(os.path.join(native.ROOT, "include", header)).read()
    return sorted(set(re.findall(r"\b(%s_\w+)\s*\(" % prefix, src)) - {prefix + "_ctx"})


def test_parser_and_decoder_entry_points_exported(native_lib):
    """libav1r.so carries the host parser (include/av1p.h) and the whole-decoder C-ABI
    (include/av1dec.h) too, so one library is the drop-in; libav1p.so is the parser alone."""
    for header, prefix in (("av1p.h", "av1p"), ("av1dec.h", "av1d")):
        names = _declared(header, prefix)
        assert names, header
        for n in names:
            assert hasattr(native_lib, n), n
    assert sorted(native.PARSE_EXPORTS) == _declared("av1p.h", "av1p")
    plib = C.CDLL(native.build_parser())
    for n in native.PARSE_EXPORTS:
        assert hasattr(plib, n), n
    # the C++ facade (YamiAv1::Decoder, Yami::YuvFrame) is exported with C++ linkage
    import subprocess
    syms = subprocess.run(["nm", "-DC", native.LIB], capture_output=True, text=True).stdout
    for s in ("YamiAv1::Decoder::decode(unsigned char*, unsigned long)", "YamiAv1::Decoder::getOutput()",
              "Yami::YuvFrame::create(int, int)"):
        assert s in syms, s


def test_cli_usage_without_device():
    """The av1dec CLI (tests/Av1Dec.cpp's counterpart) is built next to the library and
    rejects a bad command line before touching any device."""
    import subprocess
    r = subprocess.run([native.CLI], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "usage" in r.stderr
    r = subprocess.run([native.CLI, "-i", "/nonexistent.ivf"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "can't open" in r.stderr


def test_cycle_source_bounds(native_lib):
    """The in-memory cycling source (av1r_cycle_next) checks its stream index, and the
    pipeline refuses it without a frame budget (it never ends) -- both before any device use."""
    frames = batchfile.load(golden.batch_path("64x64"))
    row = (C.c_void_p * 1)(C.cast(frames[0].byref(), C.c_void_p).value)
    table = (C.c_void_p * 1)(C.cast(row, C.c_void_p).value)
    count = (C.c_int * 1)(1)
    pos = (C.c_int64 * 1)(0)
    cyc = native.Cycle(C.cast(table, C.c_void_p).value, count, pos, 1)
    out = C.c_void_p()
    assert native_lib.av1r_cycle_next(C.byref(cyc), 0, C.byref(out)) == 0 and out.value == row[0]
    assert pos[0] == 1
    assert native_lib.av1r_cycle_next(C.byref(cyc), 1, C.byref(out)) == abi.AV1R_E_INVALID
    assert native_lib.av1r_cycle_next(C.byref(cyc), -1, C.byref(out)) == abi.AV1R_E_INVALID
    src = native.StreamSource(C.cast(native_lib.av1r_cycle_next, C.c_void_p).value,
                              C.cast(C.pointer(cyc), C.c_void_p).value, 1)
    ctxs = (C.c_void_p * 1)(1)  # never dereferenced: rejected first
    st = native.PipelineStats()
    assert native_lib.av1r_pipeline_run(ctxs, 1, C.byref(src), 0, 0, 1, C.byref(st)) == abi.AV1R_E_INVALID
    ctxs2 = (C.c_void_p * 2)(1, 1)
    assert native_lib.av1r_pipeline_run(ctxs2, 2, C.byref(src), 5, 0, 1, C.byref(st)) == abi.AV1R_E_INVALID
    # the persistent pipeline: a cycle source with fewer streams than contexts, null
    # arguments, a step without a pipeline -- all refused before any thread or device use
    p = C.c_void_p()
    assert native_lib.av1r_pipeline_open(ctxs2, 2, C.byref(src), 0, 1, C.byref(p)) == abi.AV1R_E_INVALID
    assert native_lib.av1r_pipeline_open(ctxs, 1, C.byref(src), 0, 1, None) == abi.AV1R_E_INVALID
    assert native_lib.av1r_pipeline_open(None, 1, C.byref(src), 0, 1, C.byref(p)) == abi.AV1R_E_INVALID
    assert native_lib.av1r_pipeline_step(None, 5, C.byref(st)) == abi.AV1R_E_INVALID
    counts = (C.c_int64 * 1)()
    assert native_lib.av1r_pipeline_launched(None, counts, 1) == abi.AV1R_E_INVALID
    native_lib.av1r_pipeline_close(None)  # a no-op


def test_lean_intra_constants_match_the_tables():
    """intra_fast.h restates two spec tables as immediates (the smooth weights of sides 4,
    8, 16 and the intra edge kernel): they must equal av1r_tables.h / av1r_consts.h."""
    root = native.ROOT
    src = open(os.path.join(root, "av1dec_amd", "csrc", "intra_fast.h")).read()
    tab = open(os.path.join(root, "include", "av1r_tables.h")).read()
    body = tab[tab.index("av1r_sm_weights[124]"):]
    sm = [int(v) for v in re.findall(r"\d+", body[body.index("{"):body.index("}")])][:28]
    fn = src[src.index("DEV uint32_t fi_smw"):]
    fn = fn[:fn.index("\n}")]
    words = [int(h, 16) for h in re.findall(r"0x([0-9a-f]{8})u", fn)]
    got = [(w >> (8 * b)) & 0xff for w in words for b in range(4)]
    assert got == sm  # 4: words[0]; 8: words[1..2]; 16: words[3..6]
    cst = open(os.path.join(root, "include", "av1r_consts.h")).read()
    ek = cst[cst.index("av1r_edge_kernel[3][5]"):]
    ek = [int(v) for v in re.findall(r"\d+", ek[ek.index("{"):ek.index(";")])]
    kern = [ek[5 * i:5 * i + 5] for i in range(3)]

    def sel(name, s):  # evaluate fi_ek0/1/2 of intra_fast.h for strength s
        f = src[src.index(f"DEV int {name}(int str)"):]
        expr = f[f.index("return") + 6:f.index(";")].strip()
        def tern(e):  # C's right-associative  c ? a : rest
            if "?" not in e:
                return int(e)
            c, rest = e.split("?", 1)
            a, rest = rest.split(":", 1)
            return int(a) if eval(c.replace("str", str(s)), {}) else tern(rest.strip())
        return tern(expr)
    for s in (1, 2, 3):
        k = kern[s - 1]
        assert k == k[::-1]
        assert [sel("fi_ek0", s), sel("fi_ek1", s), sel("fi_ek2", s)] == k[:3], s


# MD5 over the packed bytes of the first 40 fixture streams and six synthetic 1080p frames
# (tools/pack_digest.py 40).  Round 5 checked the fused map walks of build_schedule against
# the separate ones (AV1R_PACK_FUSED, since removed) with it.  Round 6 found the sections'
# padding unwritten (heap contents travelled; under MALLOC_PERTURB_ the digest changed from
# run to run) and zeroes it; pruning the library's measured-slower paths left the packed
# bytes unchanged; the tiny items' marks (WorkItem::hflags) then changed them.  A change that alters the packed layout on purpose updates it here.
PACK_DIGEST = "0eadecd12144b13b31485d6a55c679fb 82"  # (digest, frames)


def test_pack_digest_unchanged():
    """The packed batches (av1r_pack, host only) of the fixture streams and the bench's
    synthetic frames are byte-identical to the committed digest."""
    import subprocess
    import sys
    tool = os.path.join(native.ROOT, "tools", "pack_digest.py")
    # (glibc fills fresh allocations with the perturb byte: unwritten bytes would change it)
    for perturb in ("17", "165"):
        out = subprocess.run([sys.executable, tool, "40"], capture_output=True, text=True, timeout=600,
                             env=dict(os.environ, MALLOC_PERTURB_=perturb)).stdout.split()
        assert out == PACK_DIGEST.split(), perturb


def test_validation_palette_window_keyed_on_the_tbs_own_block(native_lib):
    """A transform block's palette map window is checked against the block its `block` field
    names (what build_schedule and the device follow), not against the block whose TB range it
    sits in: a TB in a non-palette block's range that names a palette block elsewhere in the
    frame must be rejected (it would read outside that block's colour map)."""
    import numpy as np
    fr = batchfile.load(golden.batch_path("Halo_426x240_1frames_intrabc"))[0]
    err = C.create_string_buffer(256)
    assert native_lib.av1r_check_batch(C.cast(fr.byref(), C.c_void_p), None, err, 256) == 0
    blk = np.frombuffer(fr.sec["blocks"].tobytes(), abi.BLOCK_DTYPE)
    tb = np.frombuffer(fr.sec["tbs"].tobytes(), abi.TB_DTYPE).copy()
    pal = [i for i in range(len(blk)) if blk["palette_size_y"][i] and not blk["flags"][i] & 1]  # AV1R_BLK_INTER
    assert pal
    p = pal[0]
    px, py = int(blk["mi_col"][p]) * 4, int(blk["mi_row"][p]) * 4
    # a luma TB of a non-palette block far from the palette block
    far = [i for i in range(len(tb)) if tb["plane"][i] == 0 and not blk["palette_size_y"][tb["block"][i]]
           and (abs(int(tb["x"][i]) - px) > 64 or abs(int(tb["y"][i]) - py) > 64)]
    assert far
    tb["block"][far[0]] = p
    secs = dict(fr.sec)
    secs["tbs"] = tb.view(np.uint8).ravel()
    bad = batchfile.Frame(secs)
    assert native_lib.av1r_check_batch(C.cast(bad.byref(), C.c_void_p), None, err, 256) == abi.AV1R_E_INVALID
    assert b"palette map window" in err.value


def test_shipped_code_has_no_ashr_pk_u8(tmp_path):
    """Regression guard: hipcc (ROCm 7.2) folded a clamp + byte packing into
    v_ashr_pk_u8_i32, whose destination's upper half gfx950 leaves as it was while the compiler
    assumed it zero -- loop restoration came out wrong at every x % 4 == 2 pixel.  No gfx950
    code object of libav1r.so may contain that instruction."""
    import shutil
    import subprocess
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        import pytest
        pytest.skip("llvm-objdump not present")
    lib = tmp_path / "libav1r.so"
    shutil.copy(native.LIB, lib)
    subprocess.run([objdump, "--offloading", str(lib)], cwd=tmp_path, capture_output=True, check=True, timeout=120)
    objs = sorted(p for p in tmp_path.iterdir() if p.name.endswith("gfx950"))
    assert objs, "no gfx950 code object in libav1r.so"
    for o in objs:
        dis = subprocess.run([objdump, "-d", str(o)], capture_output=True, text=True, check=True, timeout=300).stdout
        assert "k_flow" in dis or "k_lr" in dis or "k_inter" in dis
        assert "v_ashr_pk_u8" not in dis, o.name


def test_frame_layout_describes_one_linear_read_back(native_lib):
    """av1r_frame_layout (include/av1r.h): the library's frame layout, which a read-back
    destination copies to get one linear transfer per frame (the ring sink's slots).  Plane
    offsets and strides are 256-byte aligned, planes do not overlap, and `span` reaches the
    last visible byte of plane 2; a bad size is refused.  Host-only: no device needed."""
    st, off, span = (C.c_int * 3)(), (C.c_size_t * 3)(), C.c_size_t()
    for w, h in ((1920, 1080), (3840, 2160), (226, 226), (64, 66), (16, 16)):
        assert native_lib.av1r_frame_layout(w, h, st, off, C.byref(span)) == 0
        assert off[0] == 0 and all(o % 256 == 0 for o in off) and all(s % 256 == 0 for s in st)
        assert st[0] >= w and st[1] == st[2] >= w >> 1
        assert off[1] >= st[0] * h and off[2] >= off[1] + st[1] * (h >> 1)  # no overlap
        assert span.value == off[2] + st[2] * ((h >> 1) - 1) + (w >> 1)
    assert native_lib.av1r_frame_layout(0, 1080, st, off, C.byref(span)) == abi.AV1R_E_INVALID
    assert native_lib.av1r_frame_layout(1920, 1 << 20, st, off, C.byref(span)) == abi.AV1R_E_INVALID


def test_pack_layout_verified():
    """av1r_pack under AV1R_PACK_VERIFY=1 (read once per process, hence the child): every
    section of the packed frame placed in order inside the buffer, and every device
    transform-block record and coefficient (16-bit and 32-bit forms) read back as the kernels
    read them equal to the batch's -- on streams with large levels (quantizer-00), palette,
    loop restoration and intra block copy."""
    import subprocess
    import sys
    code = r"""
import sys
sys.path.insert(0, %r)
sys.path.insert(0, %r)
import golden
from av1dec_amd import Decoder, batchfile, native
l = native.lib()
n = 0
for s in ("av1-1-b8-00-quantizer-00", "av1-1-b8-06-mfmv", "av1-1-b8-04-cdfupdate", "Halo_426x240_1frames_intrabc", "64x64"):
    for fr in batchfile.load(golden.batch_path(s)):
        if fr.show_existing:
            continue
        p = Decoder.pack(fr)
        Decoder.free_packed(p)
        n += 1
print("packed", n)
""" % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, AV1R_PACK_VERIFY="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "packed" in r.stdout



def test_validation_rejects_ext_flags_that_disagree_with_the_block(native_lib):
    """The device reaches an inter-intra block's TB range and a local warp through the
    block's palette_off (DevBlock): validate() must reject INTERINTRA / LOCAL_VALID on an
    intra block, INTERINTRA on an inter block whose ref_frame[1] is not INTRA_FRAME, and an
    inter-intra block (ref_frame[1] == INTRA_FRAME) without the flag."""
    import numpy as np
    INTER, INTERINTRA, LOCAL_VALID = 1, 1 << 5, 1 << 7
    err = C.create_string_buffer(256)
    fr = batchfile.load(golden.batch_path("av1-1-b8-06-mfmv"))[1]
    assert native_lib.av1r_check_batch(C.cast(fr.byref(), C.c_void_p), None, err, 256) == 0
    blk0 = np.frombuffer(fr.sec["blocks"].tobytes(), abi.BLOCK_DTYPE)

    def check(mut):
        blk = blk0.copy()
        mut(blk)
        secs = dict(fr.sec)
        secs["blocks"] = blk.view(np.uint8).ravel()
        bad = batchfile.Frame(secs)  # (kept alive across the call: byref points into it)
        return native_lib.av1r_check_batch(C.cast(bad.byref(), C.c_void_p), None, err, 256)

    intra = [i for i in range(len(blk0)) if not blk0["flags"][i] & INTER]
    inter = [i for i in range(len(blk0)) if blk0["flags"][i] & INTER and blk0["ref_frame"][i][1] != 0
             and 3 <= blk0["mi_size"][i] <= 9]  # BLOCK_8X8 .. BLOCK_32X32
    assert intra and inter

    def set_flag(i, f):
        def m(b):
            b["flags"][i] |= f
        return m
    assert check(set_flag(intra[0], LOCAL_VALID)) == abi.AV1R_E_INVALID
    assert check(set_flag(intra[0], INTERINTRA)) == abi.AV1R_E_INVALID
    assert check(set_flag(inter[0], INTERINTRA)) == abi.AV1R_E_INVALID
    assert b"INTERINTRA" in err.value

    def make_ii_unflagged(b):
        b["ref_frame"][inter[0]][1] = 0
        b["flags"][inter[0]] &= 0xFFFFFFFF ^ INTERINTRA
    assert check(make_ii_unflagged) == abi.AV1R_E_INVALID

