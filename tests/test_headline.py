"""The exact paths bench.py times, at the headline configuration, checked frame by frame.

* cycle: bench.py's headline -- the native pipeline (av1r_pipeline_open, then steps, as the
  bench keeps it open across priming, warmup and the timed window) over the in-memory batches of the bench's
  own 8 synthetic 1080p streams (bench.rank_streams seeds), GOP phases staggered as the bench
  staggers them, bench.host_workers() packing threads, the pipeline's default look-ahead,
  deep (key) frames launched alone, batch re-ordering -- for one whole GOP per stream (every
  stream's key frame inside), outputs KEPT: every output frame's MD5 equals the CPU oracle's
  on the same batches.  The reference semantics is Decoder::decodeFrame per frame
  (decoder/Av1Decoder.cpp:128-192).
* ivf: bench.py's configs[4] leg -- av1r_pipeline_run over the IVF source, 8 writer streams
  (tools/bsw 1080p_s1, seeds 0x5eed1000 + stream, the bench's ivf_frames), parsed and packed
  on native threads: stream 0's first frames equal the REFERENCE decoder's MD5
  (tests/golden/bsw.json, the same seed), and every frame of every stream equals the oracle
  fed by the host parser."""
import hashlib
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))
sys.path.insert(0, os.path.join(ROOT, "tools", "bsw"))


def _frame_md5(planes):
    return b"".join(hashlib.md5(p.tobytes()).digest() for p in planes)


def _oracle_md5s(frames):
    import pyoracle
    o = pyoracle.Oracle(keep_stages=False)
    out = []
    try:
        for f in frames:
            o.decode_frame(f)
            while o.output_pending():
                out.append(_frame_md5(o.get_output()))
    finally:
        o.close()
    return out


def test_headline_helpers_are_the_bench_ones():
    """CPU: the parity tests below build their workload with bench.py's own functions."""
    import bench
    assert bench.rank_stream_ids(0, 8) == list(range(8))
    assert bench.gop_offsets(8, 60) == [j * 60 // 8 for j in range(8)]
    assert bench.host_workers() >= 1


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_gpu_headline_cycle_path_matches_oracle():
    import bench
    from av1dec_amd import Decoder
    from av1dec_amd.pipeline import NativePipeline
    S, F = 8, 60
    streams = bench.rank_streams("1080p", 0, S, F)
    with ThreadPoolExecutor(min(S, 16)) as ex:
        ref = [ex.submit(_oracle_md5s, s) for s in streams]  # CPU, meanwhile
        decs = [Decoder(0, keep_stages=False) for _ in range(S)]
        try:
            # bench.py: stream j brought alone to its GOP phase j * F / S (untimed setup)
            pp = bench.StreamScheduler(decs, F, streams=streams, workers=1)
            pp.stagger()
            pp.close()
            pos = list(pp.pos)
            pos0 = list(pos)
            # bench.py's pipeline: kept open across the priming pass, the warmup and the timed
            # window (here: three steps covering one GOP), workers packing ahead throughout
            pl = NativePipeline(decs, streams, pos, depth=0, workers=bench.host_workers())
            try:
                frames = sum(pl.step(k)["frames"] for k in (5, 20, F - 25))
                pos = pl.positions()
            finally:
                pl.close()
            assert frames == S * F
            assert pos == [p + F for p in pos0]
            keys = sum(1 for j in range(S) for t in range(pos0[j], pos0[j] + F) if streams[j][t % F].hdr.frame_type == 0)
            assert keys == S  # one whole GOP per stream: every key frame ran in the pipeline
            got = [[] for _ in range(S)]
            for j, d in enumerate(decs):
                while d.output_pending():
                    got[j].append(_frame_md5(d.get_output()))
        finally:
            for d in decs:
                d.close()
        ref = [r.result() for r in ref]
    for j in range(S):
        off = bench.gop_offsets(S, F)[j]
        assert len(got[j]) == off + F
        for k, m in enumerate(got[j]):
            assert m == ref[j][k % F], f"stream {j} output {k} (frame {k % F})"


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_gpu_headline_ivf_path_matches_reference_and_oracle():
    import bench
    from av1dec_amd import Decoder, parser
    from av1dec_amd.pipeline import run_native
    S = 8
    frames = 24  # bench.py --ivf-frames default
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "bsw.json")))["1080p_s1"]
    assert gold["seed"] == 0x5EED1000  # bench stream 0 is the stream the reference decoded
    streams = bench.ivf_streams(0, S, frames)
    with ThreadPoolExecutor(min(S, 16)) as ex:
        ref = [ex.submit(lambda s: _oracle_md5s(parser.Parser().decode_ivf(s)), s) for s in streams]
        decs = [Decoder(0, keep_stages=False) for _ in range(S)]
        try:
            st = run_native(decs, "ivf", streams)  # as bench.ivf_leg calls it
            assert st["frames"] == S * frames
            outs = [[] for _ in range(S)]
            for j, d in enumerate(decs):
                while d.output_pending():
                    outs[j].append(d.get_output())
        finally:
            for d in decs:
                d.close()
        ref = [r.result() for r in ref]
    md = hashlib.md5()
    for planes in outs[0][:gold["frames"]]:
        for p in planes:
            md.update(p.tobytes())
    assert md.hexdigest() == gold["md5"]  # the reference decoder's own output
    for j in range(S):
        assert len(outs[j]) == frames
        for k, planes in enumerate(outs[j]):
            assert _frame_md5(planes) == ref[j][k], f"stream {j} frame {k}"


class _DigestSink:
    """An output sink (av1dec_amd.pipeline.ArraySink) that keeps each delivered frame's MD5s."""

    def __init__(self, n):
        from av1dec_amd.pipeline import ArraySink
        self.sink = ArraySink(n)
        self.md5 = [[] for _ in range(n)]
        orig = self.sink._deliver

        def deliver(user, stream, status):
            orig(user, stream, status)
            self.md5[stream].append(_frame_md5(self.sink.frames[stream].pop()))
        self.sink._deliver = deliver
        from av1dec_amd import native
        import ctypes as C
        self.sink._del = native.SINK_DELIVER(deliver)
        self.sink.s.deliver = C.cast(self.sink._del, C.c_void_p).value


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_gpu_headline_async_delivery_matches_oracle():
    """bench.py's output leg: the headline pipeline with frame delivery (av1r_pipeline_set_output):
    every shown frame's read-back starts on the context's read-back stream as soon as its batch is
    launched and lands while later batches decode (av1r_get_output_async / av1r_output_query),
    delivered in order per stream -- over one whole GOP of the 8 bench streams (key frames
    included), every delivered frame equals the CPU oracle.  Reference: Decoder::getOutput
    (decoder/Av1Decoder.cpp:203-211) drained after every unit (tests/Av1Dec.cpp:216-220)."""
    import bench
    from av1dec_amd import Decoder
    from av1dec_amd.pipeline import NativePipeline
    S, F = 8, 60
    streams = bench.rank_streams("1080p", 0, S, F)
    with ThreadPoolExecutor(min(S, 16)) as ex:
        ref = [ex.submit(_oracle_md5s, s) for s in streams]
        decs = [Decoder(0, keep_stages=False) for _ in range(S)]
        ds = _DigestSink(S)
        try:
            pos0 = [bench.gop_offsets(S, F)[j] for j in range(S)]
            # every stream starts at its key frame here, then runs one GOP + its phase offset
            pl = NativePipeline(decs, streams, [0] * S, depth=0, workers=bench.host_workers())
            try:
                pl.set_output(ds.sink)
                n = sum(pl.step(k)["frames"] for k in (7, 23, F - 30))
                assert n == S * F
                pl.set_output(None)
            finally:
                pl.close()
            assert all(d.output_pending() == 0 for d in decs)  # everything was delivered
        finally:
            for d in decs:
                d.close()
        ref = [r.result() for r in ref]
    assert pos0  # (phases are exercised by the cycle test above)
    for j in range(S):
        assert ds.sink.status[j] == [0] * F
        assert ds.md5[j] == ref[j], f"stream {j}"


@pytest.mark.gpu
def test_gpu_get_output_async_and_prefetch_match_oracle():
    """av1r_get_output_async per frame (tickets polled, then waited for out of order across
    streams) and av1r_set_output_prefetch (the Yami facade's mode: read-backs started at launch,
    av1r_get_output waits for the staged copy) both return the oracle's frames, on a conformance
    stream and two synthetic 1080p streams."""
    import bench
    import golden
    import numpy as np
    from av1dec_amd import Decoder, batchfile
    import ctypes
    sets = [batchfile.load(golden.batch_path("av1-1-b8-06-mfmv"))] + bench.rank_streams("1080p", 0, 2, 6)
    for frames in sets:
        ref = _oracle_md5s(frames)
        # async: queue every frame's read-back, then wait in reverse order
        d = Decoder(0, keep_stages=False)
        try:
            tickets = []
            for f in frames:
                d.decode_frame(f)
                while d.output_pending():
                    w, h = d.output_size()
                    planes = (np.empty((h, w), np.uint8), np.empty((h >> 1, w >> 1), np.uint8),
                              np.empty((h >> 1, w >> 1), np.uint8))
                    tickets.append(d.get_output_async(*planes))
            assert d.get_output_async(*planes) is None
            got = [None] * len(tickets)
            for k in reversed(range(len(tickets))):
                tickets[k].ready()
                got[k] = _frame_md5(tickets[k].wait())
            assert got == ref
        finally:
            d.close()
        # async into pinned host memory (hipHostMalloc: a DMA straight into the caller's
        # planes), waited for in order
        from av1dec_amd.native import PinnedBuffer
        d = Decoder(0, keep_stages=False)
        bufs = []
        try:
            tickets = []
            for f in frames:
                d.decode_frame(f)
                while d.output_pending():
                    w, h = d.output_size()
                    cw, ch = (w + 1) >> 1, (h + 1) >> 1
                    b = PinnedBuffer(w * h + 2 * cw * ch)
                    bufs.append(b)
                    a = np.ctypeslib.as_array((ctypes.c_uint8 * b.n).from_address(b.ptr.value))
                    a[:] = 0xA5  # stale bytes must not survive
                    tickets.append(d.get_output_async(a[:w * h].reshape(h, w), a[w * h:w * h + cw * ch].reshape(ch, cw),
                                                      a[w * h + cw * ch:].reshape(ch, cw)))
            got = [_frame_md5(t.wait()) for t in tickets]
            assert got == ref
        finally:
            d.close()
            for b in bufs:
                b.close()
        # prefetch
        d = Decoder(0, keep_stages=False)
        try:
            assert d.l.av1r_set_output_prefetch(d.c, 1) == 0
            got = []
            for f in frames:
                d.decode_frame(f)
                if d.output_pending() > 1:
                    got.append(_frame_md5(d.get_output()))
            while d.output_pending():
                got.append(_frame_md5(d.get_output()))
            assert got == ref
        finally:
            d.close()


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_gpu_ring_sink_frames_match_oracle():
    """The bench's output sink (av1r_ring_sink_create: pinned slots in rotation): two synthetic
    1080p streams through the native pipeline, 12 frames each (key frame
    first), every frame left in the ring equals the CPU oracle's."""
    import bench
    from av1dec_amd import Decoder
    from av1dec_amd.pipeline import NativePipeline, RingSink
    S, F = 2, 12
    streams = bench.rank_streams("1080p", 0, S, F)
    ref = [_oracle_md5s(s) for s in streams]
    decs = [Decoder(0, keep_stages=False) for _ in range(S)]
    sink = RingSink(S, 1920, 1080)
    try:
        pl = NativePipeline(decs, streams, [0] * S, depth=0, workers=bench.host_workers())
        try:
            pl.set_output(sink)
            assert pl.step(F)["frames"] == S * F
            pl.set_output(None)
        finally:
            pl.close()
        for j in range(S):
            assert sink.delivered(j) == F
            assert [_frame_md5(sink.frame(j, k)) for k in range(F)] == ref[j], f"stream {j}"
    finally:
        sink.close()
        for d in decs:
            d.close()


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_gpu_sink_delivers_show_existing_frames():
    """Frame delivery of show_existing_frame units in shared launches (advisor r04): the writer's
    cif_hidden stream (hidden frames, then show_existing_frame units) on four contexts at
    staggered phases through the native pipeline with an output sink, so that a stream's
    show-existing entry is applied after its frames ran in batches led by other contexts, and
    sometimes while it led a batch itself.  A read-back ticket must wait for the launch that
    wrote the shown frame (FrameBuf::wMeta), not for the context's last launch: every delivered
    frame equals the CPU oracle's.  Reference: Decoder::showExistingFrame
    (decoder/Av1Decoder.cpp:158-169)."""
    import bench
    from av1dec_amd import Decoder, parser
    from av1dec_amd.pipeline import NativePipeline
    import pybsw
    import pyoracle
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "bsw.json")))["cif_hidden"]
    frames = parser.Parser().decode_ivf(pybsw.stream_ivf("cif_hidden", seed=gold["seed"]))
    F, S = len(frames), 4
    assert any(f.show_existing for f in frames)
    # the oracle over two cycles: the outputs each entry produces (frame 0 refreshes every slot)
    o = pyoracle.Oracle(keep_stages=False)
    per_entry = []
    try:
        for f in frames + frames:
            o.decode_frame(f)
            outs = []
            while o.output_pending():
                outs.append(_frame_md5(o.get_output()))
            per_entry.append(outs)
    finally:
        o.close()
    offs = [1 + j * (F - 2) // S for j in range(S)]
    decs = [Decoder(0, keep_stages=False) for _ in range(S)]
    ds = _DigestSink(S)
    try:
        for j, d in enumerate(decs):  # each stream alone to its phase, outputs drained
            for f in frames[:offs[j]]:
                d.decode_frame(f)
            while d.output_pending():
                d.get_output()
        pl = NativePipeline(decs, [frames] * S, offs, depth=0, workers=bench.host_workers())
        try:
            pl.set_output(ds.sink)
            assert pl.step(F)["frames"] == S * F
            pl.set_output(None)
        finally:
            pl.close()
        assert all(d.output_pending() == 0 for d in decs)
    finally:
        for d in decs:
            d.close()
    for j in range(S):
        want = [m for e in range(offs[j], offs[j] + F) for m in per_entry[e]]
        assert ds.sink.status[j] == [0] * len(want)
        assert ds.md5[j] == want, f"stream {j}"
