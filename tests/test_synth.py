"""Synthetic bench workload (tools/synth): deterministic, valid batches, and -- on the
GPU -- bit-exact with the CPU oracle at the bench's full 1080p size and the 4K 4x2-tile
configuration (BASELINE.json configs[2], configs[3])."""
import ctypes as C
import hashlib

import pytest

import pyoracle
import pysynth
from av1dec_amd import Decoder


def test_generator_deterministic():
    a = pysynth.stream(352, 288, 3, 11)
    b = pysynth.stream(352, 288, 3, 11)
    c = pysynth.stream(352, 288, 3, 12)
    assert [f.to_bytes() for f in a] == [f.to_bytes() for f in b]
    assert a[1].to_bytes() != c[1].to_bytes()


@pytest.mark.parametrize("w,h,tiles", [(352, 288, (1, 1)), (640, 360, (2, 2))])
def test_generated_batches_validate(native_lib, w, h, tiles):
    err = C.create_string_buffer(256)
    for f in pysynth.stream(w, h, 4, 5, tiles=tiles):
        lv = C.c_int()
        assert native_lib.av1r_check_batch(C.cast(f.byref(), C.c_void_p), C.byref(lv), err, 256) == 0, err.value
        assert lv.value >= 1


def test_oracle_runs_synthetic():
    o = pyoracle.Oracle(keep_stages=False)
    for f in pysynth.stream(352, 288, 3, 3):
        o.decode_frame(f)
    n = 0
    while o.output_pending():
        y, u, v = o.get_output()
        assert y.shape == (288, 352)
        n += 1
    assert n == 3


def compare_gpu_oracle(frames, stages=True):
    d = Decoder(0, keep_stages=stages)
    o = pyoracle.Oracle(keep_stages=stages)
    for i, f in enumerate(frames):
        d.decode_frame(f)
        o.decode_frame(f)
        if stages:
            for st in range(4):
                a = d.read_stage(st)
                b = o.read_stage(st)
                for p in range(3):
                    assert (a[p] == b[p]).all(), f"frame {i} stage {st} plane {p}"
    n = 0
    while o.output_pending():
        a = d.get_output()
        b = o.get_output()
        for x, y in zip(a, b):
            assert hashlib.md5(x.tobytes()).digest() == hashlib.md5(y.tobytes()).digest(), f"output {n}"
        n += 1
    assert d.output_pending() == 0
    d.close()
    return n


@pytest.mark.gpu
def test_gpu_synth_cif_all_stages():
    assert compare_gpu_oracle(pysynth.stream(352, 288, 8, 21)) == 8


@pytest.mark.gpu
def test_gpu_synth_1080p():
    assert compare_gpu_oracle(pysynth.stream(1920, 1080, 4, 0x5EED0001), stages=True) == 4


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_gpu_synth_4k_tiles():
    """BASELINE configs[3]: 3840x2160, 4x2 uniform tiles, every stage of 4 frames (key + 3
    inter) bit-exact with the oracle."""
    assert compare_gpu_oracle(pysynth.stream(3840, 2160, 4, 0x5EED0002, tiles=(4, 2)), stages=True) == 4


@pytest.mark.gpu
def test_gpu_prepared_path_matches_streaming():
    frames = pysynth.stream(640, 360, 5, 9)
    d1 = Decoder(0)
    d2 = Decoder(0)
    hs = [d2.prepare(f) for f in frames]
    for f, hd in zip(frames, hs):
        d1.decode_frame(f)
        d2.decode_prepared(hd)
    while d1.output_pending():
        for x, y in zip(d1.get_output(), d2.get_output()):
            assert (x == y).all()


@pytest.mark.gpu
@pytest.mark.parametrize("sizes", [[(352, 288)] * 3, [(640, 360), (352, 288), (416, 240), (640, 360)]])
def test_gpu_batched_streams_match_oracle(sizes):
    """av1r_decode_prepared_batch: independent streams (different seeds, and different
    frame sizes in the second case) in shared launches, each bit-exact with the oracle."""
    nfr = 4
    streams = [pysynth.stream(w, h, nfr, 100 + i) for i, (w, h) in enumerate(sizes)]
    decs = [Decoder(0, keep_stages=False) for _ in streams]
    handles = [[d.prepare(f) for f in s] for d, s in zip(decs, streams)]
    for t in range(nfr):
        Decoder.decode_prepared_batch(decs, [h[t] for h in handles])
    for d, s in zip(decs, streams):
        o = pyoracle.Oracle(keep_stages=False)
        for f in s:
            o.decode_frame(f)
        n = 0
        while o.output_pending():
            for x, y in zip(d.get_output(), o.get_output()):
                assert (x == y).all(), f"stream output {n}"
            n += 1
        assert n == nfr
    for d, hs in zip(decs, handles):
        for hd in hs:
            d.release_prepared(hd)
        d.close()


@pytest.mark.gpu
def test_gpu_concurrent_contexts_match_oracle():
    """Independent decoders on their own HIP streams, frames issued round-robin with no
    synchronisation in between: their k_flow launches share the device's flow stream
    (concurrent k_flow grids could starve each other) and each stays bit-exact."""
    nfr = 3
    streams = [pysynth.stream(w, h, nfr, 300 + i) for i, (w, h) in enumerate([(640, 360), (352, 288), (640, 360), (416, 240)])]
    decs = [Decoder(0, keep_stages=False) for _ in streams]
    for t in range(nfr):
        for d, s in zip(decs, streams):
            d.decode_frame(s[t])
    for d, s in zip(decs, streams):
        o = pyoracle.Oracle(keep_stages=False)
        for f in s:
            o.decode_frame(f)
        n = 0
        while o.output_pending():
            for x, y in zip(d.get_output(), o.get_output()):
                assert (x == y).all(), f"output {n}"
            n += 1
        assert n == nfr
        d.close()


@pytest.mark.gpu
def test_gpu_threaded_contexts_match_oracle():
    """One host thread per decoder (contexts are independent: validation, scheduling,
    upload and launches run concurrently; k_flow launches share the device's flow chain):
    every stream stays bit-exact."""
    import threading
    nfr = 4
    dims = [(640, 360), (352, 288), (640, 360), (416, 240), (1280, 720), (640, 360), (352, 288), (704, 576)]
    streams = [pysynth.stream(w, h, nfr, 400 + i) for i, (w, h) in enumerate(dims)]
    decs = [Decoder(0, keep_stages=False) for _ in streams]
    errs = []

    def feed(d, s):  # from the very first frame: key frames of all threads overlap
        try:
            for f in s:
                d.decode_frame(f)
            d.synchronize()
        except Exception as e:
            errs.append(e)
    th = [threading.Thread(target=feed, args=(d, s)) for d, s in zip(decs, streams)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    for d, s in zip(decs, streams):
        o = pyoracle.Oracle(keep_stages=False)
        for f in s:
            o.decode_frame(f)
        n = 0
        while o.output_pending():
            for x, y in zip(d.get_output(), o.get_output()):
                assert (x == y).all(), f"output {n}"
            n += 1
        assert n == nfr
        d.close()


def _mixed_lr(frame):
    """The frame with 32-px loop-restoration units on luma, alternating Wiener / self-guided
    by column, so every 64-px k_lr tile mixes both types (its two-round path)."""
    import numpy as np
    from av1dec_amd import abi, batchfile
    sec = dict(frame.sec)
    h = abi.FrameHdr.from_buffer_copy(sec["hdr"].tobytes())
    units = np.frombuffer(sec["lr"].tobytes(), dtype=abi.LR_DTYPE).copy()
    wie = units[units["type"] == 1][0]
    sgr = units[units["type"] == 2][0]
    rows = max((h.frame_height + 16) // 32, 1)
    cols = max((h.frame_width + 16) // 32, 1)
    new = np.zeros(rows * cols, dtype=abi.LR_DTYPE)
    for c in range(cols):
        new[c::cols] = wie if c % 2 == 0 else sgr
    h.lr_type[0] = 3  # switchable
    h.lr_unit_size[0] = 32
    h.lr_unit_rows[0], h.lr_unit_cols[0], h.lr_unit_off[0] = rows, cols, len(units)
    sec["lr"] = np.concatenate([units, new]).view(np.uint8)
    sec["hdr"] = np.frombuffer(bytes(h), dtype=np.uint8).copy()
    return batchfile.Frame(sec)


@pytest.mark.gpu
def test_gpu_lr_mixed_unit_tiles():
    """k_lr tiles whose units mix Wiener and self-guided (the LDS they share is used in two
    rounds): every stage equals the oracle's."""
    frames = [_mixed_lr(f) for f in pysynth.stream(640, 360, 2, 0x5EED0077)]
    d = Decoder(0, keep_stages=True)
    o = pyoracle.Oracle(keep_stages=True)
    for i, f in enumerate(frames):
        assert f.hdr.uses_lr
        d.decode_frame(f)
        o.decode_frame(f)
        for p, (a, b) in enumerate(zip(d.read_stage(3), o.read_stage(3))):
            assert (a == b).all(), f"frame {i} LR plane {p}"
    d.close()


@pytest.mark.gpu
def test_gpu_level_schedule_synth_1080p():
    """The level-launch schedule on the bench's 1080p stream (stages checked)."""
    frames = pysynth.stream(1920, 1080, 3, 0x5EED0003)
    d = Decoder(0, keep_stages=True)
    d.set_schedule(0)
    o = pyoracle.Oracle(keep_stages=True)
    for i, f in enumerate(frames):
        d.decode_frame(f)
        o.decode_frame(f)
        for st in range(4):
            for p, (a, b) in enumerate(zip(d.read_stage(st), o.read_stage(st))):
                assert (a == b).all(), f"frame {i} stage {st} plane {p}"
    d.close()


@pytest.mark.gpu
def test_gpu_flow_timeout_surfaces_as_device_error():
    """A k_flow wait that gives up (forced: one poll allowed) must never hand out its frame
    as AV1R_OK: get_output / synchronize report AV1R_E_DEVICE for every frame of the stream
    from the failed launch on (they may reference it), for every context of the batch."""
    from av1dec_amd.decoder import BackendError
    frames = [pysynth.stream(640, 360, 3, 0x5EED0099 + i) for i in range(2)]
    decs = [Decoder(0, keep_stages=False) for _ in frames]
    for d in decs:  # the bound of the launching context applies (batch lead, or a key frame's own)
        d.set_flow_spins(1)
    handles = [[d.prepare(f) for f in s] for d, s in zip(decs, frames)]
    for t in range(3):
        Decoder.decode_prepared_batch(decs, [h[t] for h in handles])
    for d in decs:
        with pytest.raises(BackendError, match=r"\(-3\)"):
            d.synchronize()
        d.synchronize()  # reported once
        n = 0
        while d.output_pending():
            with pytest.raises(BackendError, match=r"\(-3\)"):
                d.get_output()
            n += 1
        assert n == 3
    # the same stream with the default bound decodes bit-exact again from its key frame
    for d in decs:
        d.set_flow_spins(0)
    for t in range(3):
        Decoder.decode_prepared_batch(decs, [h[t] for h in handles])
    o = pyoracle.Oracle(keep_stages=False)
    for f in frames[0]:
        o.decode_frame(f)
    while o.output_pending():
        for x, y in zip(decs[0].get_output(), o.get_output()):
            assert (x == y).all()
    for d, hs in zip(decs, handles):
        for hd in hs:
            d.release_prepared(hd)
        d.close()


def _oracle_md5s(frames):
    o = pyoracle.Oracle(keep_stages=False)
    out = []
    for f in frames:
        o.decode_frame(f)
        while o.output_pending():
            out.append(b"".join(hashlib.md5(p.tobytes()).digest() for p in o.get_output()))
    o.close()
    return out


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_gpu_bench_workload_matches_oracle():
    """The exact workload bench.py times: 8 synthetic 1080p streams with the bench's seeds
    through av1r_decode_prepared_batch, each stream offset to its own GOP phase, one whole
    GOP (key frame included) per stream -- every output frame bit-exact with the oracle."""
    from concurrent.futures import ThreadPoolExecutor
    import bench
    S, F = 8, 60
    W, H, tiles, seed = bench.CONFIGS["1080p"]
    with ThreadPoolExecutor(8) as ex:
        streams = list(ex.map(lambda j: pysynth.stream(W, H, F, bench.stream_seed(seed, j), sb128=True, tiles=tiles),
                              range(S)))
        ref = ex.submit(lambda: list(ex.map(_oracle_md5s, streams)))
        decs = [Decoder(0, keep_stages=False) for _ in range(S)]
        handles = [[d.prepare(f) for f in fr] for d, fr in zip(decs, streams)]
        ss = bench.StreamScheduler(decs, F, handles=handles)
        ss.stagger()
        got = [[] for _ in range(S)]
        keys = 0
        for _ in range(F // 4):
            keys += sum(1 for j, t in ss.run(4) if t == 0)
            for j, d in enumerate(decs):
                while d.output_pending():
                    got[j].append(b"".join(hashlib.md5(p.tobytes()).digest() for p in d.get_output()))
        ref = ref.result()
    assert keys >= S - 1  # the timed-style window holds key frames (each launched alone)
    for j in range(S):
        off = bench.gop_offsets(S, F)[j]
        assert len(got[j]) == off + F
        for k, m in enumerate(got[j]):
            assert m == ref[j][k % F], f"stream {j} output {k} (frame {k % F})"
    for d, hs in zip(decs, handles):
        for hd in hs:
            d.release_prepared(hd)
        d.close()


@pytest.mark.gpu
def test_gpu_packed_batches_match_oracle():
    """av1r_pack + av1r_decode_packed_batch (flow-only schedules, uploads from pinned memory
    on the copy stream), with an intra-block-copy frame (level schedule) in the same batch as
    flow-only frames: every output bit-exact with the oracle."""
    import golden
    from av1dec_amd import batchfile
    streams = [pysynth.stream(w, h, 4, 500 + i) for i, (w, h) in enumerate([(640, 360), (352, 288), (416, 240)])]
    streams.append(batchfile.load(golden.batch_path("Halo_426x240_1frames_intrabc")))
    decs = [Decoder(0, keep_stages=False) for _ in streams]
    for t in range(4):
        members = [i for i, s in enumerate(streams) if t < len(s)]
        packs = [Decoder.pack(streams[i][t]) for i in members]
        Decoder.decode_packed_batch([decs[i] for i in members], packs)
        for p in packs:
            Decoder.free_packed(p)
    for d, s in zip(decs, streams):
        ref = _oracle_md5s(s)
        n = 0
        while d.output_pending():
            assert b"".join(hashlib.md5(p.tobytes()).digest() for p in d.get_output()) == ref[n], f"output {n}"
            n += 1
        assert n == len(ref)
        d.close()


@pytest.mark.gpu
def test_gpu_pack_pipeline_matches_oracle():
    """bench.py's headline path (StreamScheduler: packing threads ahead of the launches,
    stream GOP phases staggered, key frames launched alone while the other streams' batches
    go on) on 4 small streams over two GOPs: bit-exact with the oracle."""
    import bench
    S, F = 4, 6
    streams = [pysynth.stream(640, 360, F, 600 + j) for j in range(S)]
    decs = [Decoder(0, keep_stages=False) for _ in range(S)]
    pp = bench.StreamScheduler(decs, F, streams=streams, workers=3)
    pp.stagger()
    pp.run(2 * F)
    pp.close()
    for j, (d, s) in enumerate(zip(decs, streams)):
        ref = _oracle_md5s(s)
        got = []
        while d.output_pending():
            got.append(b"".join(hashlib.md5(p.tobytes()).digest() for p in d.get_output()))
        assert len(got) == bench.gop_offsets(S, F)[j] + 2 * F
        for k, m in enumerate(got):
            assert m == ref[k % F], f"stream {j} output {k}"
        d.close()


@pytest.mark.gpu
def test_gpu_native_pipeline_matches_oracle():
    """bench.py's headline path since round 2 (av1r_pipeline_run over in-memory batches: a
    native packing thread per stream, GOP phases staggered, key frames alone) on 4 small
    streams over two GOPs, in three runs that continue each other: bit-exact with the oracle."""
    import bench
    from av1dec_amd.pipeline import run_native
    S, F = 4, 6
    streams = [pysynth.stream(640, 360, F, 700 + j) for j in range(S)]
    decs = [Decoder(0, keep_stages=False) for _ in range(S)]
    pp = bench.StreamScheduler(decs, F, streams=streams, workers=1)
    pp.stagger()
    pp.close()
    pos = list(pp.pos)
    for k in (F, 1, F - 1):
        st = run_native(decs, "cycle", streams, pos, max_frames=k)
        assert st["frames"] == S * k
    for j, (d, s) in enumerate(zip(decs, streams)):
        ref = _oracle_md5s(s)
        got = []
        while d.output_pending():
            got.append(b"".join(hashlib.md5(p.tobytes()).digest() for p in d.get_output()))
        assert len(got) == bench.gop_offsets(S, F)[j] + 2 * F
        for k, m in enumerate(got):
            assert m == ref[k % F], f"stream {j} output {k}"
        d.close()
