"""Synthetic AV1 bitstreams (tools/bsw) decoded three ways.

tests/golden/bsw.json holds, per configuration of tools/bsw/pybsw.CONFIGS, the SHA-256 of
the stream the writer produces and the MD5 of the REFERENCE decoder's output on it
(tools/bsw_golden.py, run in the build container with the reference built from its own
sources).  The configurations cover what the conformance set never executes (SURVEY §8c
K6): 1080p and 4K, multi-tile (2x2, 4x2), 64x64 superblocks, loop-filter sharpness and
delta updates, delta_q / delta_lf (single and multi), translation / rotzoom / affine
global motion, switchable loop restoration, periodic key frames.

* CPU: the writer is deterministic (SHA-256), exact (every temporal unit re-parsed by an
  independent parser reproduces the writer's batches), and bitstream -> host parser -> CPU
  oracle reproduces the reference's MD5.
* GPU: bitstream -> host parser -> libav1r (C-ABI) reproduces the reference's MD5, and so
  does the av1dec command-line decoder (the YamiAv1::Decoder facade)."""
import hashlib
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "bsw"))
import pybsw  # noqa: E402

GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "bsw.json")))
NAMES = sorted(GOLD)
BIG = {"1080p_s1", "4k_s2_tiles4x2"}


def stream(name):
    g = GOLD[name]
    return pybsw.stream_ivf(name, seed=g["seed"])


def test_golden_covers_every_config():
    assert set(GOLD) == set(pybsw.CONFIGS)


def test_hidden_and_show_existing_units():
    """cif_hidden's units carry hidden frames (show_frame = 0) and show_existing_frame units:
    the parser yields one more frame batch per hidden frame and one show-existing entry per
    such unit, and exactly one shown frame per unit."""
    from av1dec_amd import parser
    frames = parser.Parser().decode_ivf(stream("cif_hidden"))
    hidden = [f for f in frames if not f.show_existing and not f.hdr.show_frame]
    shown_existing = [f for f in frames if f.show_existing]
    assert len(hidden) == len(shown_existing) == 3
    assert len(frames) - len(hidden) == GOLD["cif_hidden"]["frames"]


@pytest.mark.parametrize("name", NAMES)
def test_writer_is_exact(name):
    """Every unit re-parsed by a second parser gives the writer's own frame batches."""
    n = 2 if name in BIG else None
    pybsw.write(name=name, frames=n, verify=True, seed=GOLD[name]["seed"])


@pytest.mark.parametrize("name", NAMES)
def test_writer_is_deterministic(name):
    data = stream(name)
    assert len(data) == GOLD[name]["bytes"]
    assert pybsw.sha256(data) == GOLD[name]["sha256"]


def _md5_of(frames, dec):
    md = hashlib.md5()
    for fr in frames:
        dec.decode_frame(fr)
        while dec.output_pending():
            for p in dec.get_output():
                md.update(p.tobytes())
    return md.hexdigest()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_md5(name):
    """Bitstream -> host parser -> CPU restatement == the reference decoder's MD5."""
    import pyoracle
    from av1dec_amd import parser
    frames = parser.Parser().decode_ivf(stream(name))
    assert sum(1 for f in frames if f.show_existing or f.hdr.show_frame) == GOLD[name]["frames"]  # shown frames
    o = pyoracle.Oracle(keep_stages=False)
    try:
        assert _md5_of(frames, o) == GOLD[name]["md5"]
    finally:
        o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_matches_reference_md5(native_lib, name):
    """Bitstream -> host parser -> HIP backend (C-ABI) == the reference decoder's MD5."""
    from av1dec_amd import Decoder, parser
    frames = parser.Parser().decode_ivf(stream(name))
    d = Decoder(0)
    try:
        assert _md5_of(frames, d) == GOLD[name]["md5"]
    finally:
        d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["1080p_s1", "640x360_tiles2x2_sb64", "cif_gm_affine_sb64"])
def test_gpu_cli_matches_reference_md5(native_lib, name, tmp_path):
    """The av1dec CLI (YamiAv1::Decoder facade, the reference's tests/Av1Dec.cpp flow)."""
    from av1dec_amd import native
    f = tmp_path / f"{name}.ivf"
    f.write_bytes(stream(name))
    r = subprocess.run([native.CLI, "-i", str(f), "-md5"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-500:]
    assert re.search(r"md5=([0-9a-f]{32})", r.stdout + r.stderr).group(1) == GOLD[name]["md5"]


@pytest.mark.gpu
def test_gpu_ivf_pipeline_matches_reference_md5(native_lib):
    """The bench's configs[4] path (av1dec_amd.pipeline: a parse+pack thread per stream,
    shared launches) on streams of three sizes at once, outputs kept: every stream's MD5
    equals the reference's."""
    from av1dec_amd import Decoder
    from av1dec_amd.pipeline import IvfPipeline
    names = ["1080p_s1", "cif_s1", "640x360_tiles2x2_sb64", "odd_416x234_key3", "cif_hidden"]
    decs = [Decoder(0) for _ in names]
    try:
        outs = [[] for _ in names]
        pl = IvfPipeline(decs, [stream(n) for n in names])
        pl.run()
        for d, o in zip(decs, outs):
            while d.output_pending():
                o.append(d.get_output())
        for n, o in zip(names, outs):
            md = hashlib.md5()
            for planes in o:
                for p in planes:
                    md.update(p.tobytes())
            assert md.hexdigest() == GOLD[n]["md5"], n
    finally:
        for d in decs:
            d.close()


@pytest.mark.gpu
def test_gpu_native_pipeline_ivf_matches_reference_md5(native_lib):
    """av1r_pipeline_run over the IVF source (native producer threads, the bench's
    ivf_end_to_end path) on five streams of different sizes, outputs kept.  cif_hidden carries
    hidden frames and show_existing_frame units: the pipeline's show-existing entries
    (av1r_show_existing, ordered by sequence number across the workers) in output order."""
    from av1dec_amd import Decoder
    from av1dec_amd.pipeline import run_native
    names = ["1080p_s1", "cif_gm_rotzoom", "640x360_tiles2x2_sb64", "odd_416x234_key3", "cif_hidden"]
    decs = [Decoder(0) for _ in names]
    try:
        st = run_native(decs, "ivf", [stream(n) for n in names])
        from av1dec_amd import parser  # decoded frames: shown, hidden and show-existing entries
        assert st["frames"] == sum(len(parser.Parser().decode_ivf(stream(n))) for n in names)
        for n, d in zip(names, decs):
            md = hashlib.md5()
            while d.output_pending():
                for p in d.get_output():
                    md.update(p.tobytes())
            assert md.hexdigest() == GOLD[n]["md5"], n
    finally:
        for d in decs:
            d.close()


def test_flow_schedules_hold_their_invariants():
    """Every packed frame of five writer streams (av1r_pack, the pipeline's flow-only
    schedule) through the host-side schedule check (AV1R_SCHED_CHECK=1, schedule_check in
    av1r_host.cpp): indices in range, every listed or edge-granule dependency in an earlier
    k_flow group, residual tiles inside the residual buffer.  Host only."""
    code = (
        "import sys, ctypes as C\n"
        f"sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tools', 'bsw')!r})\n"
        "import pybsw, json\n"
        "from av1dec_amd import native, parser\n"
        "l = native.lib()\n"
        f"gold = json.load(open({os.path.join(ROOT, 'tests', 'golden', 'bsw.json')!r}))\n"
        "for n in ['cif_s1', '640x360_tiles2x2_sb64', 'odd_416x234_key3', 'cif_hidden', 'cif_gm_affine_sb64']:\n"
        "    for f in parser.Parser(mode_info=False).decode_ivf(pybsw.stream_ivf(n, seed=gold[n]['seed'])):\n"
        "        pk = C.c_void_p()\n"
        "        assert l.av1r_pack(C.cast(f.byref(), C.c_void_p), C.byref(pk)) == 0\n"
        "        l.av1r_packed_free(pk)\n")
    env = dict(os.environ, AV1R_SCHED_CHECK="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stderr.splitlines() if x.startswith("av1r sched check:")]
    summaries = [x for x in lines if "violations" in x]
    assert summaries, r.stderr[-2000:]
    assert all(x.endswith(" 0 violations") for x in summaries), "\n".join(lines[:30])
