"""The arithmetic the inter sub-pixel passes rely on (recon.hip: hfilt_pk / vfilt_pk / hpass /
pred_win4), checked exhaustively on the CPU against the spec tables the kernels read.

hpass computes a horizontal output as two v_dot4_i32_i8 of the taps HALVED (signed bytes) with
the pixels biased to signed bytes (p ^ 0x80 = p - 128):

    sum f[u] * p[u] = 2 * sum (f[u] / 2) * (p[u] - 128) + 128 * 128

which holds only if every tap is even, every halved tap fits a signed byte and every filter
sums to 128 (the reference's blockSubPixelPredict, InterPredict.cpp:340-362, multiplies the
unhalved taps).  pred_win4 takes the vertical taps as int16 pairs for v_dot2_i32_i16.
"""
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def subpel_filters():
    text = open(os.path.join(ROOT, "include", "av1r_tables.h")).read()
    m = re.search(r"av1r_subpel_filters\[768\]\s*=\s*\{([^}]*)\}", text)
    vals = np.array([int(v) for v in m.group(1).replace("\n", " ").split(",") if v.strip()], dtype=np.int64)
    assert vals.size == 768
    return vals.reshape(96, 8)  # (set * 16 + phase, tap)


def test_taps_even_halved_fit_signed_bytes_and_sum_128():
    f = subpel_filters()
    assert (f % 2 == 0).all()
    h = f // 2
    assert h.min() >= -128 and h.max() <= 127
    assert (f.sum(axis=1) == 128).all()
    # vertical taps as int16 pairs (vfilt_pk): every tap fits int16
    assert f.min() >= -32768 and f.max() <= 32767


def sdot4(a, b):
    """v_dot4_i32_i8 on byte vectors already sign-interpreted."""
    return int(np.dot(a.astype(np.int64), b.astype(np.int64)))


def test_hpass_identity_every_filter_random_and_extreme_windows():
    f = subpel_filters()
    rng = np.random.default_rng(7)
    windows = [np.zeros(8, np.int64), np.full(8, 255, np.int64), np.array([0, 255] * 4, np.int64),
               np.array([255, 0] * 4, np.int64)] + [rng.integers(0, 256, 8) for _ in range(64)]
    for row in f:
        h = row // 2
        for p in windows:
            ref = int(np.dot(row, p))
            s = ((p ^ 0x80) - 128 * ((p ^ 0x80) >> 7) * 2)  # p ^ 0x80 read as a signed byte
            assert (s == p - 128).all()
            dot = sdot4(h[:4], s[:4]) + sdot4(h[4:], s[4:])
            assert 2 * dot + 16384 == ref


def test_vertical_dot2_pairs_match_the_tap_sum():
    f = subpel_filters()
    rng = np.random.default_rng(11)
    for row in f:
        for _ in range(32):
            col = rng.integers(-32768, 32768, 8)  # int16 intermediates
            pairs = sum(int(row[2 * t]) * int(col[2 * t]) + int(row[2 * t + 1]) * int(col[2 * t + 1]) for t in range(4))
            assert pairs == int(np.dot(row, col))
