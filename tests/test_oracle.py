"""The CPU oracle (oracle/av1r_oracle.c) against the REFERENCE's own outputs.

For every conformance stream the committed batches were extracted from the reference
decoder by oracle/harness/refdump.cpp, together with the MD5 of each reference stage
(reconstruction, LoopFilter, Cdef, LoopRestoration).  The oracle must reproduce every
stage hash of every frame and the whole-output MD5 listed in bits/bits.md5 (the
reference's conformance pins, testscript/conformance.py:42-91)."""
import hashlib

import pytest

import golden
import pyoracle
from av1dec_amd import batchfile

STREAMS = golden.streams()
BITS = golden.bits_md5()


def test_fixture_inventory():
    assert len(STREAMS) == 172
    for s in STREAMS:
        assert s in BITS, s


@pytest.mark.parametrize("stream", STREAMS)
def test_oracle_matches_reference(stream):
    frames = batchfile.load(golden.batch_path(stream))
    rows, out_md5 = golden.stage_hashes(stream)
    assert len(rows) == len(frames)
    o = pyoracle.Oracle(keep_stages=True)
    md = hashlib.md5()
    for i, fr in enumerate(frames):
        o.decode_frame(fr)
        if not fr.show_existing:
            for st, name in enumerate(("recon", "lf", "cdef", "lr")):
                assert pyoracle.md5_planes(o.read_stage(st)) == rows[i][3 + st], f"frame {i} {name}"
        while o.output_pending():
            for p in o.get_output():
                md.update(p.tobytes())
    assert md.hexdigest() == out_md5 == BITS[stream]
