// txfm_dev.h -- AV1 1-D inverse transforms for one lane's row/column held in registers.
//
// Restates iDct / iAdst4/8/16 / iIdentity / inverseWalshHadamardTransform
// (decoder/TransformBlock.cpp:1751-2166).  Every butterfly index, angle and bit-reversal
// is a compile-time constant after unrolling (template<int N>), so T[] lives in VGPRs
// and the cos/sin factors become immediates.
#pragma once
#include "av1r_dev.h"

namespace tx {

constexpr int kCos128[65] = {
    4096, 4095, 4091, 4085, 4076, 4065, 4052, 4036, 4017, 3996, 3973, 3948, 3920, 3889, 3857, 3822,
    3784, 3745, 3703, 3659, 3612, 3564, 3513, 3461, 3406, 3349, 3290, 3229, 3166, 3102, 3035, 2967,
    2896, 2824, 2751, 2675, 2598, 2520, 2440, 2359, 2276, 2191, 2106, 2019, 1931, 1842, 1751, 1660,
    1567, 1474, 1380, 1285, 1189, 1092, 995, 897, 799, 700, 601, 501, 401, 301, 201, 101, 0};

constexpr int cos128(int angle)
{
    return (angle & 255) <= 64 ? kCos128[angle & 255]
        : (angle & 255) <= 128 ? -kCos128[128 - (angle & 255)]
        : (angle & 255) <= 192 ? -kCos128[(angle & 255) - 128]
        : kCos128[256 - (angle & 255)];
}
constexpr int sin128(int angle) { return cos128(angle - 64); }
constexpr int brev(int numBits, int x)
{
    int t = 0;
    for (int i = 0; i < numBits; i++) t |= ((x >> i) & 1) << (numBits - 1 - i);
    return t;
}

DEV int rnd12(int x) { return (x + 2048) >> 12; }

template <int a, int b, int angle, bool flip>
DEV void B(int* T)
{
    constexpr int c = cos128(angle), s = sin128(angle);
    int x = T[a] * c - T[b] * s;
    int y = T[a] * s + T[b] * c;
    if (!flip) {
        T[a] = rnd12(x);
        T[b] = rnd12(y);
    } else {
        T[b] = rnd12(x);
        T[a] = rnd12(y);
    }
}
template <int a0, int b0, bool flip>
DEV void H(int* T, int lo, int hi)
{
    constexpr int a = flip ? b0 : a0, b = flip ? a0 : b0;
    int x = T[a], y = T[b];
    T[a] = CLIP3(lo, hi, x + y);
    T[b] = CLIP3(lo, hi, x - y);
}

// compile-time for-loop
template <int I, int N, class F>
DEV void sfor(F&& f)
{
    if constexpr (I < N) {
        f(std::integral_constant<int, I>());
        sfor<I + 1, N>(f);
    }
}

// iDct (TransformBlock.cpp:1827-1989), n = log2 size
template <int n>
DEV void idct(int* T, int r)
{
    const int lo = -(1 << (r - 1)), hi = (1 << (r - 1)) - 1;
    constexpr int cnt = 1 << n;
    {
        int c[cnt];
#pragma unroll
        for (int i = 0; i < cnt; i++) c[i] = T[i];
        sfor<0, cnt>([&](auto i) { T[i] = c[brev(n, i)]; });
    }
    if constexpr (n == 6) sfor<0, 16>([&](auto i) { B<32 + i, 63 - i, 63 - 4 * brev(4, i), false>(T); });
    if constexpr (n >= 5) sfor<0, 8>([&](auto i) { B<16 + i, 31 - i, 6 + (brev(3, 7 - i) << 3), false>(T); });
    if constexpr (n == 6) sfor<0, 16>([&](auto i) { H<32 + i * 2, 33 + i * 2, (i & 1) != 0>(T, lo, hi); });
    if constexpr (n >= 4) sfor<0, 4>([&](auto i) { B<8 + i, 15 - i, 12 + (brev(2, 3 - i) << 4), false>(T); });
    if constexpr (n >= 5) sfor<0, 8>([&](auto i) { H<16 + 2 * i, 17 + 2 * i, (i & 1) != 0>(T, lo, hi); });
    if constexpr (n == 6)
        sfor<0, 4>([&](auto i) { sfor<0, 2>([&](auto j) { B<62 - i * 4 - j, 33 + i * 4 + j, 60 - 16 * brev(2, i) + 64 * j, true>(T); }); });
    if constexpr (n >= 3) sfor<0, 2>([&](auto i) { B<4 + i, 7 - i, 56 - 32 * i, false>(T); });
    if constexpr (n >= 4) sfor<0, 4>([&](auto i) { H<8 + 2 * i, 9 + 2 * i, (i & 1) != 0>(T, lo, hi); });
    if constexpr (n >= 5)
        sfor<0, 2>([&](auto i) { sfor<0, 2>([&](auto j) { B<30 - 4 * i - j, 17 + 4 * i + j, 24 + (j << 6) + ((1 - i) << 5), true>(T); }); });
    if constexpr (n == 6)
        sfor<0, 8>([&](auto i) { sfor<0, 2>([&](auto j) { H<32 + i * 4 + j, 35 + i * 4 - j, (i & 1) != 0>(T, lo, hi); }); });
    sfor<0, 2>([&](auto i) { B<2 * i, 2 * i + 1, 32 + 16 * i, (1 - i) != 0>(T); });
    if constexpr (n >= 3) sfor<0, 2>([&](auto i) { H<4 + 2 * i, 5 + 2 * i, i != 0>(T, lo, hi); });
    if constexpr (n >= 4) sfor<0, 2>([&](auto i) { B<14 - i, 9 + i, 48 + 64 * i, true>(T); });
    if constexpr (n >= 5)
        sfor<0, 4>([&](auto i) { sfor<0, 2>([&](auto j) { H<16 + 4 * i + j, 19 + 4 * i - j, (i & 1) != 0>(T, lo, hi); }); });
    if constexpr (n == 6)
        sfor<0, 2>([&](auto i) { sfor<0, 4>([&](auto j) { B<61 - i * 8 - j, 34 + i * 8 + j, 56 - i * 32 + (j >> 1) * 64, true>(T); }); });
    sfor<0, 2>([&](auto i) { H<i, 3 - i, false>(T, lo, hi); });
    if constexpr (n >= 3) B<6, 5, 32, true>(T);
    if constexpr (n >= 4)
        sfor<0, 2>([&](auto i) { sfor<0, 2>([&](auto j) { H<8 + 4 * i + j, 11 + 4 * i - j, i != 0>(T, lo, hi); }); });
    if constexpr (n >= 5) sfor<0, 4>([&](auto i) { B<29 - i, 18 + i, 48 + (i >> 1) * 64, true>(T); });
    if constexpr (n == 6)
        sfor<0, 4>([&](auto i) { sfor<0, 4>([&](auto j) { H<32 + 8 * i + j, 39 + 8 * i - j, (i & 1) != 0>(T, lo, hi); }); });
    if constexpr (n >= 3) sfor<0, 4>([&](auto i) { H<i, 7 - i, false>(T, lo, hi); });
    if constexpr (n >= 4) sfor<0, 2>([&](auto i) { B<13 - i, 10 + i, 32, true>(T); });
    if constexpr (n >= 5)
        sfor<0, 2>([&](auto i) { sfor<0, 4>([&](auto j) { H<16 + i * 8 + j, 23 + i * 8 - j, i != 0>(T, lo, hi); }); });
    if constexpr (n == 6) sfor<0, 8>([&](auto i) { B<59 - i, 36 + i, (i < 4 ? 48 : 112), true>(T); });
    if constexpr (n >= 4) sfor<0, 8>([&](auto i) { H<i, 15 - i, false>(T, lo, hi); });
    if constexpr (n >= 5) sfor<0, 4>([&](auto i) { B<27 - i, 20 + i, 32, true>(T); });
    if constexpr (n == 6)
        sfor<0, 8>([&](auto i) {
            H<32 + i, 47 - i, false>(T, lo, hi);
            H<48 + i, 63 - i, true>(T, lo, hi);
        });
    if constexpr (n >= 5) sfor<0, 16>([&](auto i) { H<i, 31 - i, false>(T, lo, hi); });
    if constexpr (n == 6) {
        sfor<0, 8>([&](auto i) { B<55 - i, 40 + i, 32, true>(T); });
        sfor<0, 32>([&](auto i) { H<i, 63 - i, false>(T, lo, hi); });
    }
}

DEV void iadst4(int* T)
{
    const int S1 = 1321, S2 = 2482, S3 = 3344, S4 = 3803;
    int s0 = S1 * T[0], s1 = S2 * T[0], s2 = S3 * T[1], s3 = S4 * T[2];
    int s4 = S1 * T[2], s5 = S2 * T[3], s6 = S4 * T[3];
    int a7 = T[0] - T[2];
    int b7 = a7 + T[3];
    s0 = s0 + s3;
    s1 = s1 - s4;
    s3 = s2;
    s2 = S3 * b7;
    s0 = s0 + s5;
    s1 = s1 - s6;
    int x0 = s0 + s3, x1 = s1 + s3, x2 = s2, x3 = s0 + s1 - s3;
    T[0] = rnd12(x0);
    T[1] = rnd12(x1);
    T[2] = rnd12(x2);
    T[3] = rnd12(x3);
}
template <int n>
DEV void adst_in_perm(int* T)
{
    constexpr int n0 = 1 << n;
    int c[n0];
#pragma unroll
    for (int i = 0; i < n0; i++) c[i] = T[i];
    sfor<0, n0>([&](auto i) { T[i] = c[(i & 1) ? (i - 1) : (n0 - i - 1)]; });
}
template <int n>
DEV void adst_out_perm(int* T)
{
    constexpr int n0 = 1 << n;
    int c[n0];
#pragma unroll
    for (int i = 0; i < n0; i++) c[i] = T[i];
    sfor<0, n0>([&](auto i) {
        constexpr int a = (i >> 3) & 1;
        constexpr int b = ((i >> 2) & 1) ^ ((i >> 3) & 1);
        constexpr int cc = ((i >> 1) & 1) ^ ((i >> 2) & 1);
        constexpr int d = (i & 1) ^ ((i >> 1) & 1);
        constexpr int idx = ((d << 3) | (cc << 2) | (b << 1) | a) >> (4 - n);
        T[i] = (i & 1) ? -c[idx] : c[idx];
    });
}
DEV void iadst8(int* T, int r)
{
    const int lo = -(1 << (r - 1)), hi = (1 << (r - 1)) - 1;
    adst_in_perm<3>(T);
    sfor<0, 4>([&](auto i) { B<2 * i, 2 * i + 1, 60 - 16 * i, true>(T); });
    sfor<0, 4>([&](auto i) { H<i, 4 + i, false>(T, lo, hi); });
    sfor<0, 2>([&](auto i) { B<4 + 3 * i, 5 + i, 48 - 32 * i, true>(T); });
    sfor<0, 2>([&](auto i) { sfor<0, 2>([&](auto j) { H<4 * j + i, 2 + 4 * j + i, false>(T, lo, hi); }); });
    sfor<0, 2>([&](auto i) { B<2 + 4 * i, 3 + 4 * i, 32, true>(T); });
    adst_out_perm<3>(T);
}
DEV void iadst16(int* T, int r)
{
    const int lo = -(1 << (r - 1)), hi = (1 << (r - 1)) - 1;
    adst_in_perm<4>(T);
    sfor<0, 8>([&](auto i) { B<2 * i, 2 * i + 1, 62 - 8 * i, true>(T); });
    sfor<0, 8>([&](auto i) { H<i, 8 + i, false>(T, lo, hi); });
    sfor<0, 2>([&](auto i) {
        B<8 + 2 * i, 9 + 2 * i, 56 - 32 * i, true>(T);
        B<13 + 2 * i, 12 + 2 * i, 8 + 32 * i, true>(T);
    });
    sfor<0, 4>([&](auto i) { sfor<0, 2>([&](auto j) { H<8 * j + i, 4 + 8 * j + i, false>(T, lo, hi); }); });
    sfor<0, 2>([&](auto i) { sfor<0, 2>([&](auto j) { B<4 + 8 * j + 3 * i, 5 + 8 * j + i, 48 - 32 * i, true>(T); }); });
    sfor<0, 2>([&](auto i) { sfor<0, 4>([&](auto j) { H<4 * j + i, 2 + 4 * j + i, false>(T, lo, hi); }); });
    sfor<0, 4>([&](auto i) { B<2 + 4 * i, 3 + 4 * i, 32, true>(T); });
    adst_out_perm<4>(T);
}
template <int n>
DEV void iidentity(int* T)
{
#pragma unroll
    for (int i = 0; i < (1 << n); i++) {
        if constexpr (n == 2) T[i] = rnd12(T[i] * 5793);
        else if constexpr (n == 3) T[i] = T[i] * 2;
        else if constexpr (n == 4) T[i] = rnd12(T[i] * 11586);
        else if constexpr (n == 5) T[i] = T[i] * 4;
    }
}
DEV void iwht(int* T, int shift)
{
    int a = T[0] >> shift, c = T[1] >> shift, d = T[2] >> shift, b = T[3] >> shift;
    a += c;
    d -= b;
    int e = (a - d) >> 1;
    b = e - b;
    c = e - c;
    a -= b;
    d += c;
    T[0] = a;
    T[1] = b;
    T[2] = c;
    T[3] = d;
}

// kind: 0 DCT, 1 ADST, 2 identity, 3 WHT (lossless)
template <int n>
DEV void run1d(int* T, int kind, int r, int whtShift)
{
    if (kind == 0) {
        idct<n>(T, r);
    } else if (kind == 1) {
        if constexpr (n == 2) iadst4(T);
        else if constexpr (n == 3) iadst8(T, r);
        else if constexpr (n == 4) iadst16(T, r);
    } else if (kind == 2) {
        iidentity<n>(T);
    } else {
        if constexpr (n == 2) iwht(T, whtShift);
    }
}

DEV int row_kind(int t)
{
    if (t == AV1R_DCT_DCT || t == AV1R_ADST_DCT || t == AV1R_FLIPADST_DCT || t == AV1R_H_DCT) return 0;
    if (t == AV1R_DCT_ADST || t == AV1R_ADST_ADST || t == AV1R_DCT_FLIPADST || t == AV1R_FLIPADST_FLIPADST
        || t == AV1R_ADST_FLIPADST || t == AV1R_FLIPADST_ADST || t == AV1R_H_ADST || t == AV1R_H_FLIPADST)
        return 1;
    return 2;
}
DEV int col_kind(int t)
{
    if (t == AV1R_DCT_DCT || t == AV1R_DCT_ADST || t == AV1R_DCT_FLIPADST || t == AV1R_V_DCT) return 0;
    if (t == AV1R_ADST_DCT || t == AV1R_ADST_ADST || t == AV1R_FLIPADST_DCT || t == AV1R_FLIPADST_FLIPADST
        || t == AV1R_ADST_FLIPADST || t == AV1R_FLIPADST_ADST || t == AV1R_V_ADST || t == AV1R_V_FLIPADST)
        return 1;
    return 2;
}

}  // namespace tx
