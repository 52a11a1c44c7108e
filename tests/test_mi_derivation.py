"""The mode-info grid is a function of the blocks and transform blocks (batch ABI v2).

The library no longer uploads av1r_frame_batch.mi: k_mi (filters.hip) rebuilds it on the
device -- zero outside the frame, each block's mode info over its 4x4 units, each transform
block's size over the units it covers (TransformBlock.cpp:2444-2454).  This restates that
derivation on the host and checks it against the grid the reference's own parse produced
for every conformance fixture, and against the synthetic generator's grids (inside the
frame: the generator initialises the units no block reaches differently, and nothing reads
them)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))

import golden  # noqa: E402
from av1dec_amd import abi, batchfile  # noqa: E402

TX_W = [4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64]
TX_H = [4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16]
NW = [1, 1, 2, 2, 2, 4, 4, 4, 8, 8, 8, 16, 16, 16, 32, 32, 1, 4, 2, 8, 4, 16]
NH = [1, 2, 1, 2, 4, 2, 4, 8, 4, 8, 16, 8, 16, 32, 16, 32, 4, 1, 8, 2, 16, 4]


def derive_mi(fr):
    h = fr.hdr
    S, R = h.mi_stride, h.mi_rows_alloc
    mi = np.zeros(S * R, dtype=abi.MI_DTYPE).reshape(R, S)
    for b in fr.sec["blocks"].view(abi.BLOCK_DTYPE):
        r, c, bs = int(b["mi_row"]), int(b["mi_col"]), int(b["mi_size"])
        v = mi[r:r + NH[bs], c:c + NW[bs]]
        v["mv"] = b["mv"]
        v["ref_frame"] = b["ref_frame"]
        v["mi_size"] = bs
        v["y_mode"] = b["y_mode"]
        v["filt"] = b["filt"]
        v["flags"] = (1 if b["flags"] & (1 << 16) else 0) | (2 if b["flags"] & 1 else 0)
        v["delta_lf"] = b["delta_lf"]
        v["uv_mode"] = b["uv_mode"]
    for t in fr.sec["tbs"].view(abi.TB_DTYPE):
        p, sub = int(t["plane"]), (1 if t["plane"] else 0)
        row, col = (int(t["y"]) << sub) >> 2, (int(t["x"]) << sub) >> 2
        hh, ww = (TX_H[t["tx_size"]] >> 2) << sub, (TX_W[t["tx_size"]] >> 2) << sub
        mi[row:row + hh, col:col + ww]["lf_tx"][..., p] = t["tx_size"]
    return mi


@pytest.mark.parametrize("stream", golden.streams())
def test_derived_grid_equals_reference_grid(stream):
    for k, fr in enumerate(batchfile.load(golden.batch_path(stream))):
        if fr.show_existing:
            continue
        got = derive_mi(fr).reshape(-1).view(np.uint8)
        assert np.array_equal(got, fr.sec["mi"]), f"{stream} frame {k}"


def test_derived_grid_equals_synthetic_grid_inside_the_frame():
    import pysynth
    for w, h, seed in ((192, 128, 11), (1920, 1080, 0x5EED1000)):
        for fr in pysynth.stream(w, h, 2, seed, sb128=True):
            got = derive_mi(fr)
            ref = fr.sec["mi"].view(abi.MI_DTYPE).reshape(got.shape)
            H, W = fr.hdr.mi_rows, fr.hdr.mi_cols
            assert np.array_equal(got[:H, :W], ref[:H, :W])
