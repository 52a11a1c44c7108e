"""HIP backend parity on an MI355X: every stage of every frame of all 172 conformance
streams must equal the REFERENCE's stage MD5s (extracted by oracle/harness/refdump.cpp),
and the whole decoded output must equal bits/bits.md5.  Calls go through the C-ABI."""
import hashlib

import pytest

import golden
from av1dec_amd import Decoder, abi, batchfile

STREAMS = golden.streams()
BITS = golden.bits_md5()

@pytest.fixture(scope="module")
def dev(native_lib):
    d = Decoder(0, keep_stages=True)
    yield d
    d.close()


def run_stream(stream, check_stages=True, schedule=1):
    frames = batchfile.load(golden.batch_path(stream))
    rows, out_md5 = golden.stage_hashes(stream)
    d = Decoder(0, keep_stages=check_stages)
    d.set_schedule(schedule)
    md = hashlib.md5()
    bad = []
    for i, fr in enumerate(frames):
        d.decode_frame(fr)
        if check_stages and not fr.show_existing:
            for st, name in enumerate(("recon", "lf", "cdef", "lr")):
                m = hashlib.md5()
                for p in d.read_stage(st):
                    m.update(p.tobytes())
                if m.hexdigest() != rows[i][3 + st]:
                    bad.append(f"frame {i} {name}")
                    break
        while d.output_pending():
            for p in d.get_output():
                md.update(p.tobytes())
    d.close()
    return bad, md.hexdigest(), out_md5


@pytest.mark.gpu
@pytest.mark.parametrize("stream", STREAMS)
def test_gpu_matches_reference(stream):
    bad, got, out_md5 = run_stream(stream)
    assert not bad, bad[:3]
    assert got == out_md5 == BITS[stream]


@pytest.mark.gpu
@pytest.mark.parametrize("stream", STREAMS)
def test_gpu_level_schedule_matches_reference(stream):
    # the level-launch schedule (the fallback for intra block copy frames) on every stream
    bad, got, out_md5 = run_stream(stream, check_stages=False, schedule=0)
    assert got == out_md5 == BITS[stream]


@pytest.mark.gpu
def test_gpu_tile_split_api():
    # frame_begin/submit_tile/frame_end with the frame's blocks split in two "tiles"
    import numpy as np
    frames = batchfile.load(golden.batch_path("av1-1-b8-06-mfmv"))
    d1 = Decoder(0)
    d2 = Decoder(0)
    for fr in frames:
        d1.decode_frame(fr)
        n = fr.n_blocks
        if n < 2 or fr.show_existing:
            d2.decode_frame(fr)
            continue
        split_tiles(d2, fr)
    while d1.output_pending():
        a = d1.get_output()
        b = d2.get_output()
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


def split_tiles(dec, fr):
    """Split a frame's blocks into two 'tiles' with tile-local indices and offsets."""
    import numpy as np
    bt = np.frombuffer(fr.sec["blocks"].tobytes(), abi.BLOCK_DTYPE).copy()
    tt = np.frombuffer(fr.sec["tbs"].tobytes(), abi.TB_DTYPE).copy()
    coefs = np.frombuffer(fr.sec["coefs"].tobytes(), np.uint32)
    pal = fr.sec["palette"]
    nb = bt.shape[0]
    half = nb // 2
    t_split = int(bt["first_tb"][half])
    c_split = int(tt["coef_off"][t_split]) if t_split < tt.shape[0] else coefs.size
    has_pal = (bt["palette_size_y"].astype(int) + bt["palette_size_uv"]) > 0
    later = [int(bt["palette_off"][i]) for i in range(half, nb) if has_pal[i]]
    p_split = later[0] if later else pal.size
    tiles = []
    for b0, b1, t0, t1, c0, c1, p0, p1 in ((0, half, 0, t_split, 0, c_split, 0, p_split),
                                           (half, nb, t_split, tt.shape[0], c_split, coefs.size, p_split, pal.size)):
        bb = bt[b0:b1].copy()
        bb["first_tb"] -= t0
        bb["palette_off"] = np.where(has_pal[b0:b1], bb["palette_off"] - p0, 0)
        tb = tt[t0:t1].copy()
        tb["block"] -= b0
        tb["coef_off"] -= c0
        secs = dict(fr.sec)
        secs["blocks"] = bb.view(np.uint8).ravel()
        secs["tbs"] = tb.view(np.uint8).ravel()
        secs["coefs"] = coefs[c0:c1].view(np.uint8).copy()
        secs["palette"] = pal[p0:p1].copy()
        tiles.append(batchfile.Frame(secs))
    dec.decode_tiles(fr, tiles)


@pytest.mark.gpu
def test_gpu_ref_release():
    """av1r_ref_release empties slots: the key frame still decodes and reads back equal to an
    untouched decoder, an inter frame that needs an emptied slot is rejected, and a mask
    outside the 8 slots is refused."""
    import numpy as np
    from av1dec_amd.decoder import BackendError
    frames = [f for f in batchfile.load(golden.batch_path("av1-1-b8-06-mfmv")) if not f.show_existing]
    d1, d2 = Decoder(0), Decoder(0)
    d1.decode_frame(frames[0])
    d2.decode_frame(frames[0])
    d2.ref_release(0xff)
    for x, y in zip(d1.get_output(), d2.get_output()):
        assert np.array_equal(x, y)
    with pytest.raises(BackendError):
        d2.decode_frame(frames[1])
    with pytest.raises(BackendError):
        d2.ref_release(0x100)
    d1.close()
    d2.close()
