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
