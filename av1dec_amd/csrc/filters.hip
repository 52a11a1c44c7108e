// filters.hip -- in-loop post-filters for gfx950: deblocking, CDEF, loop restoration.
//
//   k_lf    one lane per 4x4 edge unit (all planes, one pass per launch): LoopFilter::
//           loop_filter_edge + sampleFilter/narrowFilter/wideFilter
//           (decoder/LoopFilter.cpp:85-289).  Edges of one pass never overlap their
//           read/write footprints (the filter length is bounded by the transform sizes
//           on both sides), so a pass is embarrassingly parallel, in place.
//   k_cdef  one workgroup per 64x64 filter region staged in LDS: Cdef::cdef_block
//           (Cdef.cpp:72-101), cdefDirection (:203-261) one lane per (block, direction),
//           cdefFilter (:158-198) one lane per pixel, into a separate output frame
//           (blocks that are skipped are copied).
//   k_lr    one workgroup per 64-column tile of a (half-)stripe, source staged in LDS:
//           LoopRestoration Wiener (LoopRestoration.cpp:247-277) and self-guided
//           (:284-479) with the stripe/unit geometry of :33-189; the 3-pixel border
//           extension (:196-198) is coordinate clamping.
#include <algorithm>
#include <cstdlib>

#include "av1r_dev.h"
#include "intra_dev.h"


// ------------------------------------------------------------------------------------
// Deblocking
// ------------------------------------------------------------------------------------
DEV int lf_level(const KParams& k, int row, int col, int plane, int pass)
{
    const av1r_frame_hdr& h = *k.hdr;
    const av1r_mi& info = mi_at(k, row, col);
    int ref = info.ref_frame[0];
    int mode = info.y_mode;
    int modeType = mode >= AV1R_NEARESTMV && mode != AV1R_GLOBALMV && mode != AV1R_GLOBAL_GLOBALMV;
    int deltaLF = h.delta_lf_multi ? info.delta_lf[plane == 0 ? pass : plane + 1] : info.delta_lf[0];
    int i = plane == 0 ? pass : plane + 1;
    int8_t l = (int8_t)CLIP3(0, 63, deltaLF + h.lf_level[i]);
    if (h.lf_delta_enabled) {
        int nShift = l >> 5;
        if (ref == AV1R_INTRA_FRAME)
            l = (int8_t)(l + (h.lf_ref_deltas[0] << nShift));
        else
            l = (int8_t)(l + (h.lf_ref_deltas[ref & 7] << nShift) + (h.lf_mode_deltas[modeType] << nShift));
        l = (int8_t)CLIP3(0, 63, l);
    }
    return l;
}

// wideFilter (LoopFilter.cpp:246-289): F[i] = Round2(sum_j tap(j) * clamp(i + j), log2Size)
// over the 2n samples around the edge; taps are 2 for |j| <= n2, else 1.
template <int n, int log2Size, int n2, class PX>
DEV void lf_wide(PX* c, int step)
{
    int v[2 * n + 2];  // v[p + n + 1] = pixel at offset p, p in [-(n + 1), n]
#pragma unroll
    for (int p = -(n + 1); p <= n; p++) v[p + n + 1] = c[step * p];
    int F[2 * n];
#pragma unroll
    for (int i = -n; i < n; i++) {
        int t = 0;
#pragma unroll
        for (int j = -n; j <= n; j++) {
            int p = CLIP3(-(n + 1), n, i + j);
            t += v[p + n + 1] * ((j <= n2 && j >= -n2) ? 2 : 1);
        }
        F[i + n] = r2(t, log2Size);
    }
#pragma unroll
    for (int i = -n; i < n; i++) c[step * i] = (uint8_t)F[i + n];
}

// sampleFilter (LoopFilter.cpp:145-289) at the edge pixel c (the first q sample), samples
// `step` apart across the edge: the frame (k_lf) or an LDS tile (k_post)
template <class PX>
DEV void lf_filter(PX* c, int step, int plane, int limit, int blimit, int thresh, int filterSize)
{
#define PP(k) c[-step * ((k) + 1)]
#define QQ(k) c[step * (k)]
    int q0 = QQ(0), q1 = QQ(1), q2 = QQ(2), q3 = QQ(3);
    int p0 = PP(0), p1 = PP(1), p2 = PP(2), p3 = PP(3);
    int hev = (iabs(p1 - p0) > thresh) | (iabs(q1 - q0) > thresh);
    int filterLen = filterSize == 4 ? 4 : (plane ? 6 : (filterSize == 8 ? 8 : 16));
    int mask = (iabs(p1 - p0) > limit) | (iabs(q1 - q0) > limit) | (iabs(p0 - q0) * 2 + iabs(p1 - q1) / 2 > blimit);
    if (filterLen >= 6) mask |= (iabs(p2 - p1) > limit) | (iabs(q2 - q1) > limit);
    if (filterLen >= 8) mask |= (iabs(p3 - p2) > limit) | (iabs(q3 - q2) > limit);
    if (mask) return;
    int flat = 0, flat2 = 0;
    if (filterSize >= 8) {
        int m = (iabs(p1 - p0) > 1) | (iabs(q1 - q0) > 1) | (iabs(p2 - p0) > 1) | (iabs(q2 - q0) > 1);
        if (filterLen >= 8) m |= (iabs(p3 - p0) > 1) | (iabs(q3 - q0) > 1);
        flat = !m;
    }
    if (filterSize >= 16) {
        int q4 = QQ(4), q5 = QQ(5), q6 = QQ(6), p4 = PP(4), p5 = PP(5), p6 = PP(6);
        int m = (iabs(p6 - p0) > 1) | (iabs(q6 - q0) > 1) | (iabs(p5 - p0) > 1) | (iabs(q5 - q0) > 1)
            | (iabs(p4 - p0) > 1) | (iabs(q4 - q0) > 1);
        flat2 = !m;
    }
    if (filterSize == 4 || !flat) {
        int ps0 = p0 - 128, ps1 = p1 - 128, qs0 = q0 - 128, qs1 = q1 - 128;
        int filter = hev ? CLIP3(-128, 127, ps1 - qs1) : 0;
        filter = CLIP3(-128, 127, filter + 3 * (qs0 - ps0));
        int filter1 = CLIP3(-128, 127, filter + 4) >> 3;
        int filter2 = CLIP3(-128, 127, filter + 3) >> 3;
        QQ(0) = (uint8_t)(CLIP3(-128, 127, qs0 - filter1) + 128);
        PP(0) = (uint8_t)(CLIP3(-128, 127, ps0 + filter2) + 128);
        if (!hev) {
            filter = r2(filter1, 1);
            QQ(1) = (uint8_t)(CLIP3(-128, 127, qs1 - filter) + 128);
            PP(1) = (uint8_t)(CLIP3(-128, 127, ps1 + filter) + 128);
        }
        return;
    }
    // wideFilter with compile-time taps (a runtime-indexed tap window would be lowered to
    // per-lane waterfall loops)
    if (filterSize >= 16 && flat2) lf_wide<6, 4, 1>(c, step);
    else if (!plane) lf_wide<3, 3, 0>(c, step);
    else lf_wide<2, 3, 1>(c, step);
#undef PP
#undef QQ
}

// lf_filter on two lines at once (two samples per 16-bit half of a dword, v_pk_* ops): the
// same decisions and arithmetic per line, every quantity fits int16 (|values| < 16384), and a
// line's filters are chosen with per-half masks (bitfield selects) instead of branches.  Each
// path reads the unfiltered samples: the paths' write masks are disjoint, and a select leaves
// the other line's samples untouched.  c: the first q sample (c[-7] .. c[6] are read).
typedef short lf2 __attribute__((ext_vector_type(2)));
DEV lf2 lf_abs(lf2 a) { return __builtin_elementwise_max(a, -a); }
DEV lf2 lf_gt(lf2 a, lf2 b) { return (b - a) >> (short)15; }  // -1 where a > b
DEV lf2 lf_clamp8(lf2 a) { return __builtin_elementwise_min(__builtin_elementwise_max(a, lf2{-128, -128}), lf2{127, 127}); }
DEV lf2 lf_sel(lf2 m, lf2 a, lf2 b) { return (a & m) | (b & ~m); }
DEV bool lf_any(lf2 m) { return (m.x | m.y) != 0; }
template <int n, int log2Size, int n2>
DEV void lf_wide2(lf2* c, lf2 m)
{
    lf2 F[2 * n];
#pragma unroll
    for (int i = -n; i < n; i++) {
        lf2 t = {0, 0};
#pragma unroll
        for (int j = -n; j <= n; j++) {
            const int p = CLIP3(-(n + 1), n, i + j);
            t += (j <= n2 && j >= -n2) ? c[p] + c[p] : c[p];
        }
        F[i + n] = (t + (short)(1 << (log2Size - 1))) >> (short)log2Size;
    }
#pragma unroll
    for (int i = -n; i < n; i++) c[i] = lf_sel(m, F[i + n], c[i]);
}
DEV void lf_filter2(lf2* c, int plane, int limit, int blimit, int thresh, int filterSize)
{
    const lf2 q0 = c[0], q1 = c[1], q2 = c[2], q3 = c[3];
    const lf2 p0 = c[-1], p1 = c[-2], p2 = c[-3], p3 = c[-4];
    const lf2 L = {(short)limit, (short)limit}, T = {(short)thresh, (short)thresh}, one = {1, 1};
    const lf2 ap1p0 = lf_abs(p1 - p0), aq1q0 = lf_abs(q1 - q0);
    const lf2 hev = lf_gt(ap1p0, T) | lf_gt(aq1q0, T);
    const int filterLen = filterSize == 4 ? 4 : (plane ? 6 : (filterSize == 8 ? 8 : 16));
    lf2 mask = lf_gt(ap1p0, L) | lf_gt(aq1q0, L) |
               lf_gt(lf_abs(p0 - q0) * (short)2 + (lf_abs(p1 - q1) >> (short)1), lf2{(short)blimit, (short)blimit});
    if (filterLen >= 6) mask |= lf_gt(lf_abs(p2 - p1), L) | lf_gt(lf_abs(q2 - q1), L);
    if (filterLen >= 8) mask |= lf_gt(lf_abs(p3 - p2), L) | lf_gt(lf_abs(q3 - q2), L);
    const lf2 apply = ~mask;
    if (!lf_any(apply)) return;
    lf2 flat = {0, 0};
    if (filterSize >= 8) {
        lf2 m = lf_gt(ap1p0, one) | lf_gt(aq1q0, one) | lf_gt(lf_abs(p2 - p0), one) | lf_gt(lf_abs(q2 - q0), one);
        if (filterLen >= 8) m |= lf_gt(lf_abs(p3 - p0), one) | lf_gt(lf_abs(q3 - q0), one);
        flat = ~m;
    }
    const lf2 narrow = apply & ~flat;
    if (lf_any(narrow)) {
        const lf2 k128 = {128, 128};
        const lf2 ps0 = p0 - k128, ps1 = p1 - k128, qs0 = q0 - k128, qs1 = q1 - k128;
        lf2 filt = lf_clamp8(ps1 - qs1) & hev;
        filt = lf_clamp8(filt + (qs0 - ps0) * (short)3);
        const lf2 f1 = lf_clamp8(filt + (short)4) >> (short)3, f2 = lf_clamp8(filt + (short)3) >> (short)3;
        c[0] = lf_sel(narrow, lf_clamp8(qs0 - f1) + k128, c[0]);
        c[-1] = lf_sel(narrow, lf_clamp8(ps0 + f2) + k128, c[-1]);
        const lf2 f = (f1 + (short)1) >> (short)1, n1 = narrow & ~hev;
        c[1] = lf_sel(n1, lf_clamp8(qs1 - f) + k128, c[1]);
        c[-2] = lf_sel(n1, lf_clamp8(ps1 + f) + k128, c[-2]);
    }
    lf2 wide = apply & flat;
    if (!lf_any(wide)) return;
    if (filterSize >= 16) {
        const lf2 q4 = c[4], q5 = c[5], q6 = c[6], p4 = c[-5], p5 = c[-6], p6 = c[-7];
        const lf2 m = lf_gt(lf_abs(p6 - p0), one) | lf_gt(lf_abs(q6 - q0), one) | lf_gt(lf_abs(p5 - p0), one) |
                      lf_gt(lf_abs(q5 - q0), one) | lf_gt(lf_abs(p4 - p0), one) | lf_gt(lf_abs(q4 - q0), one);
        const lf2 w16 = wide & ~m;
        if (lf_any(w16)) lf_wide2<6, 4, 1>(c, w16);
        wide &= m;
        if (!lf_any(wide)) return;
    }
    if (!plane) lf_wide2<3, 3, 0>(c, wide);
    else lf_wide2<2, 3, 1>(c, wide);
}

// The edge of pass `pass` (0: vertical edges, 1: horizontal) at plane position (xP, yP), a
// multiple of 4, of plane `plane` (LoopFilter::loop_filter_edge, LoopFilter.cpp:85-126, and
// the level / limit derivation, :301-359): false if no filter runs there, else its size
// and limits.  Reads only the mode-info grid.
struct LfEdge {
    int filterSize, limit, blimit, thresh;
};
// the limits of an edge of level lvl (LoopFilter.cpp:330-359)
DEV void lf_limits(const av1r_frame_hdr& hd, int lvl, LfEdge& e)
{
    const int sharp = hd.lf_sharpness;
    const int shift = sharp > 4 ? 2 : (sharp > 0 ? 1 : 0);
    e.limit = sharp > 0 ? CLIP3(1, 9 - sharp, lvl >> shift) : imax(1, lvl >> shift);
    e.blimit = 2 * (lvl + 2) + e.limit;
    e.thresh = lvl >> 4;
}
// the edge's filter size (e.filterSize) and level (returned; <= 0: no filter)
DEV int lf_edge_level(const KParams& k, int plane, int pass, int xP, int yP, LfEdge& e)
{
    const av1r_frame_hdr& hd = *k.hdr;
    const int sub = plane ? 1 : 0;
    if (plane && !hd.lf_level[plane + 1]) return 0;
    const int x = xP << sub, y = yP << sub;
    if (x < 0 || y < 0 || x >= k.frame_w || y >= k.frame_h) return 0;
    if (!pass && !x) return 0;
    if (pass && !y) return 0;
    const int dx = pass == 0, dy = pass == 1;
    const int row = (y >> 2) | sub, col = (x >> 2) | sub;
    const int prevRow = row - (dy << sub), prevCol = col - (dx << sub);
    const av1r_mi& info = mi_at(k, row, col);
    const int txSz = info.lf_tx[plane];
    const int psz = plane_bsize(info.mi_size, plane);
    const int skip = info.flags & AV1R_MI_SKIP;
    const int isIntra = info.ref_frame[0] <= AV1R_INTRA_FRAME;
    const int prevTx = mi_at(k, prevRow, prevCol).lf_tx[plane];
    // (block and transform sides are powers of two: the remainders as masks, no division)
    const int isBlockEdge = !pass ? !(xP & (av1r_num4x4w[psz] * 4 - 1)) : !(yP & (av1r_num4x4h[psz] * 4 - 1));
    const int isTxEdge = !pass ? !(xP & (av1r_tx_w[txSz] - 1)) : !(yP & (av1r_tx_h[txSz] - 1));
    if (!(isTxEdge && (isBlockEdge || !skip || isIntra))) return 0;
    const int base = !pass ? imin(av1r_tx_w[prevTx], av1r_tx_w[txSz]) : imin(av1r_tx_h[prevTx], av1r_tx_h[txSz]);
    e.filterSize = !plane ? imin(16, base) : imin(8, base);
    int lvl = lf_level(k, row, col, plane, pass);
    if (!lvl) lvl = lf_level(k, prevRow, prevCol, plane, pass);
    return lvl;
}
DEV bool lf_edge(const KParams& k, int plane, int pass, int xP, int yP, LfEdge& e)
{
    const int lvl = lf_edge_level(k, plane, pass, xP, yP, e);
    if (lvl <= 0) return false;
    lf_limits(*k.hdr, lvl, e);
    return true;
}

// The four lines of one edge unit from registers.  The unit's samples come in dwords: a
// vertical edge (pass 0) at x reads x - 4 .. x + 3 of each of its rows (x - 8 .. x + 7 for a
// 16-wide filter: its edge is >= 16 from the plane's left), a horizontal edge (pass 1) at y
// rows y - 4 .. y + 3 (y - 8 .. y + 7) of its four columns, one dword per row.  All of a
// unit's loads go out before its first filter (one memory round trip; the byte form issued
// up to 56 byte loads per unit).  Written back: the samples a filter of this size may modify
// (p1..q1 for 4 taps and chroma, p2..q2 for luma 8, p5..q5 for 16).  Rewriting an unmodified
// sample there is safe: the filter length is bounded by the transform sizes on both sides,
// so no other edge of the pass writes inside this footprint.
DEV lf2 lf_pair(uint32_t a, uint32_t b, int k)  // {byte k of a, byte k of b} (k compile-time)
{
    return __builtin_bit_cast(lf2, __builtin_amdgcn_perm(b, a, 0x0c000c00u | ((uint32_t)(4 + k) << 16) | (uint32_t)k));
}
DEV uint32_t lf_lo2(lf2 a, lf2 b)  // bytes {a.x, b.x, a.y, b.y}
{
    return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, a), 0x06020400u);
}
// The unit's pixels: the frame (k_lf, in place) or a tile staged in LDS.  x of the 32-bit
// forms is a multiple of 4, of the 16-bit forms of 2.
struct LfGlobalPx {
    uint8_t* p;
    int stride;
    DEV uint8_t* at(int x, int y) const { return p + (size_t)y * stride + x; }
    DEV uint32_t ld32(int x, int y) const { return *reinterpret_cast<const uint32_t*>(at(x, y)); }
    DEV void st32(int x, int y, uint32_t v) const { *reinterpret_cast<uint32_t*>(at(x, y)) = v; }
    DEV void st16(int x, int y, uint32_t v) const { *reinterpret_cast<uint16_t*>(at(x, y)) = (uint16_t)v; }
    DEV void st8(int x, int y, uint32_t v) const { *at(x, y) = (uint8_t)v; }
};
typedef __attribute__((address_space(3))) uint8_t lf_lds_u8;
typedef __attribute__((address_space(3))) uint16_t lf_lds_u16;
typedef __attribute__((address_space(3))) uint32_t lf_lds_u32;
struct LfLdsPx {
    lf_lds_u8* p;
    int stride;
    DEV lf_lds_u8* at(int x, int y) const { return p + y * stride + x; }
    DEV uint32_t ld32(int x, int y) const { return *reinterpret_cast<lf_lds_u32*>(at(x, y)); }
    DEV void st32(int x, int y, uint32_t v) const { *reinterpret_cast<lf_lds_u32*>(at(x, y)) = v; }
    DEV void st16(int x, int y, uint32_t v) const { *reinterpret_cast<lf_lds_u16*>(at(x, y)) = (uint16_t)v; }
    DEV void st8(int x, int y, uint32_t v) const { *at(x, y) = (uint8_t)v; }
};
template <class PX>
DEV void lf_unit(const PX& P, int plane, int pass, int xP, int yP, const LfEdge& e)
{
    const bool wide = e.filterSize == 16;
    const int n = wide ? 6 : (e.filterSize == 8 && !plane) ? 3 : 2;  // samples written per side
    if (pass == 0) {
        uint32_t d[4][4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            d[i][1] = P.ld32(xP - 4, yP + i);
            d[i][2] = P.ld32(xP, yP + i);
            d[i][0] = wide ? P.ld32(xP - 8, yP + i) : 0u;
            d[i][3] = wide ? P.ld32(xP + 4, yP + i) : 0u;
        }
        // rows (0, 1) and (2, 3) filtered as pairs: v[q] = the two rows' samples at x - 8 + q
#pragma unroll
        for (int h = 0; h < 2; h++) {
            lf2 v[16];
#pragma unroll
            for (int q = 0; q < 16; q++) v[q] = lf_pair(d[2 * h][q >> 2], d[2 * h + 1][q >> 2], q & 3);
            lf_filter2(v + 8, plane, e.limit, e.blimit, e.thresh, e.filterSize);
            // the footprint x - n .. x + n - 1 in the widest aligned stores inside it (the
            // neighbouring edges' footprints start at x - 4 - n' / x + 4 + n'': a store may
            // not spill past x - n or x + n - 1); u(q) = bytes {row a q, q + 1, row b q, q + 1}
            const int ya = yP + 2 * h, yb = ya + 1;
            auto u = [&](int q) { return lf_lo2(v[q], v[q + 1]); };
            if (n == 6) {
                const uint32_t u2 = u(2), u4 = u(4), u6 = u(6), u8 = u(8), u10 = u(10), u12 = u(12);
                P.st16(xP - 6, ya, u2);
                P.st16(xP - 6, yb, u2 >> 16);
                P.st32(xP - 4, ya, __builtin_amdgcn_perm(u6, u4, 0x05040100u));
                P.st32(xP - 4, yb, __builtin_amdgcn_perm(u6, u4, 0x07060302u));
                P.st32(xP, ya, __builtin_amdgcn_perm(u10, u8, 0x05040100u));
                P.st32(xP, yb, __builtin_amdgcn_perm(u10, u8, 0x07060302u));
                P.st16(xP + 4, ya, u12);
                P.st16(xP + 4, yb, u12 >> 16);
            } else {
                const uint32_t u6 = u(6), u8 = u(8);
                if (n == 3) {
                    P.st8(xP - 3, ya, (uint32_t)(uint16_t)v[5].x);
                    P.st8(xP - 3, yb, (uint32_t)(uint16_t)v[5].y);
                    P.st8(xP + 2, ya, (uint32_t)(uint16_t)v[10].x);
                    P.st8(xP + 2, yb, (uint32_t)(uint16_t)v[10].y);
                }
                P.st16(xP - 2, ya, u6);
                P.st16(xP - 2, yb, u6 >> 16);
                P.st16(xP, ya, u8);
                P.st16(xP, yb, u8 >> 16);
            }
        }
        return;
    }
    uint32_t d[16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const bool need = (r >= 4 && r < 12) || wide;
        d[r] = need ? P.ld32(xP, yP - 8 + r) : 0u;
    }
    // columns (0, 1) and (2, 3) filtered as pairs
    lf2 lo[16], hi[16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
        lo[r] = __builtin_bit_cast(lf2, __builtin_amdgcn_perm(0u, d[r], 0x0c010c00u));
        hi[r] = __builtin_bit_cast(lf2, __builtin_amdgcn_perm(0u, d[r], 0x0c030c02u));
    }
    lf_filter2(lo + 8, plane, e.limit, e.blimit, e.thresh, e.filterSize);
    lf_filter2(hi + 8, plane, e.limit, e.blimit, e.thresh, e.filterSize);
#pragma unroll
    for (int r = 2; r < 14; r++)
        if (r >= 8 - n && r < 8 + n)
            P.st32(xP, yP - 8 + r,
                __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, hi[r]), __builtin_bit_cast(uint32_t, lo[r]), 0x06040200u));
}

// one lane per (plane, 4x4 unit) edge of pass `pass`: the decision; then (AV1R_LF_COMPACT)
// the units that filter, packed in order to the workgroup's first lanes, one per lane
#ifndef AV1R_LF_COMPACT
#define AV1R_LF_COMPACT 1
#endif
DEV void lf_body(const KParams* kps, int pass)
{
    // (each XCD a contiguous eighth of the whole launch, i.e. about one frame; round 5: an
    // eighth of every frame's units per XCD measured within noise, r05_ab_xcd_dealing.txt)
    const uint3 wg = xcd_block();
    const KParams& k = KP(kps, wg.y);  // frame of this launch row
    const av1r_frame_hdr& hd = *k.hdr;
    if (!(hd.lf_level[0] || hd.lf_level[1])) return;  // LoopFilter::filter is skipped (the whole workgroup)
    const int nY = k.mi_rows * k.mi_cols;
    const int cCols = (k.mi_cols + 1) / 2, nC = ((k.mi_rows + 1) / 2) * cCols;
    int id = wg.x * blockDim.x + threadIdx.x;
    int plane = 0, row0 = 0, col0 = 0;
    bool valid = true;
    if (id < nY) {
        plane = 0;
        row0 = id / k.mi_cols;
        col0 = id - row0 * k.mi_cols;
    } else if (id < nY + 2 * nC) {
        int u = id - nY;
        plane = 1 + (u >= nC);
        if (u >= nC) u -= nC;
        int r = u / cCols;
        row0 = r * 2;
        col0 = (u - r * cCols) * 2;
    } else {
        valid = false;
    }
    const int sub = plane ? 1 : 0;
    const int xP = (col0 * 4) >> sub, yP = (row0 * 4) >> sub;
    // the edge's decision from the mode info, in the lane (round 5: every decision taken by a
    // separate launch ahead, k_lfcode, measured slower: 0.0116 against 0.0108 ms per 1080p
    // frame with its launch;
    // the unit's samples loaded speculatively with the mode info, before the decision:
    // 0.0119 against 0.0105, profiles/r05_ab_lf_spec.txt -- most units filter nothing)
    LfEdge e;
    const bool on = valid && lf_edge(k, plane, pass, xP, yP, e);
#if AV1R_LF_COMPACT
    // Round 6: most units filter nothing, and a wave whose few filtering lanes ran the filter
    // paid for all 64.  The filtering units of the workgroup go, in unit order (ballot +
    // per-wave prefix: rows stay contiguous for the pixel loads), to its first lanes.  A
    // pass's edges are independent -- a filter's length is bounded by the transform sizes on
    // both sides, so no edge of the pass reads or writes inside another's footprint -- so
    // the lane an edge lands on does not matter.
    __shared__ uint2 lst[256];
    __shared__ uint32_t wcnt[4];
    const uint64_t bal = __ballot(on);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) wcnt[w] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t base = 0;
    for (int i = 0; i < w; i++) base += wcnt[i];
    const uint32_t total = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    if (on) {
        const uint32_t pos = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
        lst[pos] = make_uint2((uint32_t)xP | ((uint32_t)yP << 16),
            (uint32_t)plane | ((uint32_t)e.filterSize << 2) | ((uint32_t)e.limit << 8) | ((uint32_t)e.blimit << 16) |
                ((uint32_t)e.thresh << 24));
    }
    __syncthreads();
    if (threadIdx.x >= total) return;
    const uint2 c = lst[threadIdx.x];
    LfEdge f;
    const int pl = (int)(c.y & 3);
    f.filterSize = (int)((c.y >> 2) & 31);
    f.limit = (int)((c.y >> 8) & 255);
    f.blimit = (int)((c.y >> 16) & 255);
    f.thresh = (int)(c.y >> 24);
    const DevPlane& P = k.cur.pl[pl];
    lf_unit(LfGlobalPx{P.p, P.stride}, pl, pass, (int)(c.x & 0xffff), (int)(c.x >> 16), f);
#else
    if (!on) return;
    const DevPlane& P = k.cur.pl[plane];
    lf_unit(LfGlobalPx{P.p, P.stride}, plane, pass, xP, yP, e);
#endif
}
// (forcing 6 waves per SIMD -- at most 80 VGPRs, 12 bytes of scratch -- measured no faster)
extern "C" __global__ __launch_bounds__(256) void k_lf(const KParams* kps, int pass) { lf_body(kps, pass); }

// ------------------------------------------------------------------------------------
// CDEF
// ------------------------------------------------------------------------------------
DEV int constrain(int diff, int threshold, int damping)
{
    if (!threshold) return 0;
    int adj = imax(0, damping - floor_log2(threshold));
    int ad = iabs(diff);
    int v = CLIP3(0, ad, threshold - (ad >> adj));
    return diff < 0 ? -v : v;
}

// One workgroup per 64x64 luma region (one cdef_idx, Cdef.cpp:47-55) and its two 32x32
// chroma regions.  The deblocked pixels with a 2-pixel halo are staged in LDS once (rows
// of aligned dwords away from the frame edge); the direction search runs one lane per
// (8x8 block, direction) pair summing each partial line straight from LDS; the filter
// runs two horizontally adjacent pixels per packed 16-bit operation, one 4-pixel group per
// lane and instruction.
//
// LDS banks (round 6).  Every tap read is a pair of ds_read_b32 (bank = dword mod 32, two
// 32-lane groups), so the row strides and the lane -> (row, group) maps are chosen together:
//  - luma: a half-wave holds rows r and r + 4 of one 8-row block row x the 16 dword groups
//    of the region's 64 columns; at 20 dwords per row, 4 rows are 80 = 16 (mod 32) dwords,
//    so the centre reads of the 32 lanes land on 32 distinct banks (round 5: 72-byte rows,
//    the 4 lanes of a block 2 rows apart -> 14 banks for 32 lanes, 56.7 % of LDS cycles
//    were conflicts);
//  - chroma: a half-wave holds rows r, r + 2, r + 4, r + 6 x the 8 dword groups of one
//    plane's 32 columns; at 12 dwords per row, 2 rows are 24 dwords, and {0, 24, 48, 72}
//    = {0, 24, 16, 8} (mod 32);
//  - the direction search reads each block's rows as 8-byte ds_read_b64 (bank = dword mod
//    64): blocks 8 rows apart are 160 = 32 (mod 64) dwords apart, so lanes of block rows by
//    and by + 2 read their rows in the order i ^ 4 (80 = 16 (mod 64) dwords further).
// A tap of another direction still shifts a block's lanes (per-block directions), so tap
// reads of neighbouring blocks may meet on a bank; the centre and equal-direction reads do not.
#define CD_H 2            // tap reach (Cdef_Directions)
#define CD_X 8            // LDS column of plane column x0 (dword-aligned staging from x0 - 8)
#define CD_LS 80          // luma tile: columns x0 - 8 .. x0 + 71 (20 dwords)
#define CD_LR (64 + 2 * CD_H)
#define CD_CS 48          // chroma tile: columns x0 / 2 - 8 .. x0 / 2 + 39 (12 dwords)
#define CD_CR (32 + 2 * CD_H)
struct alignas(16) CdefLds {
    uint8_t y[CD_LR][CD_LS];
    uint8_t uv[2][CD_CR][CD_CS];
    int cost[64][8];
    int16_t pri[64];               // adjusted luma primary strength
    uint8_t filt[64];              // block is filtered (not skip)
    int16_t offY[64][6], offC[64][6];  // tap offsets in the staged tiles (cdef_pair)
};

// partial[d][k] of cdefDirection (Cdef.cpp:203-261) for one line k of direction d, summed
// over the 8x8 block at (bx, by) of the staged luma tile
// (px8(i, j): the block's pixel at row i, column j, minus 128; compile-time indices)
template <int d, class F>
DEV int cdef_cost_f(const F& px8)
{
    int cost = 0;
    if (d == 2 || d == 6) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            int s = 0;
#pragma unroll
            for (int q = 0; q < 8; q++) s += d == 2 ? px8(k, q) : px8(q, k);
            cost += s * s;
        }
        return cost * av1r_cdef_div_table[8];
    }
    if (d == 0 || d == 4) {
#pragma unroll
        for (int k = 0; k < 15; k++) {
            int s = 0;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int j = d == 0 ? k - i : 7 + i - k;  // d0: k = i + j; d4: k = 7 + i - j
                if (j >= 0 && j < 8) s += px8(i, j);
            }
            cost += s * s * av1r_cdef_div_table[k < 7 ? k + 1 : (k == 7 ? 8 : 15 - k)];
        }
        return cost;
    }
    // odd directions: 11 lines; the centre 5 weigh Div_Table[8], the outer pairs 2j+2.
    // Line k of row i holds the pixels j with d1: i + j/2 == k, d3: 3 + i - j/2 == k,
    // d5: 3 - i/2 + j == k, d7: i/2 + j == k (all indices compile-time after unrolling).
#pragma unroll
    for (int k = 0; k < 11; k++) {
        int s = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (d == 1 || d == 3) {
                const int h = d == 1 ? k - i : 3 + i - k;  // j / 2
                if (h >= 0 && h <= 3) s += px8(i, 2 * h) + px8(i, 2 * h + 1);
            } else {
                const int j = d == 5 ? k - 3 + i / 2 : k - i / 2;
                if (j >= 0 && j <= 7) s += px8(i, j);
            }
        }
        const int w = (k >= 3 && k <= 7) ? av1r_cdef_div_table[8] : av1r_cdef_div_table[2 * (k < 3 ? k : 10 - k) + 2];
        cost += s * s * w;
    }
    return cost;
}
template <int d, class PX>
DEV int cdef_cost(const PX* blk, int ts)  // blk: the block's top-left pixel in a tile of row stride ts
{
    return cdef_cost_f<d>([&](int i, int j) { return (int)blk[i * ts + j] - 128; });
}

// cdefFilter (Cdef.cpp:158-198) for the four horizontally adjacent pixels at tile offset
// p (a multiple of 4) of the staged tile t (row stride ts, a multiple of 4), as two pairs
// in packed 16-bit lanes.  Each tap's four pixels come from one ds_read2_b32 and a byte
// align.  off[s * 2 + kk] = tile offset of tap kk of direction dir (s = 0), dir - 2
// (s = 1), dir + 2 (s = 2); taps at -off and +off.  `check`: the region touches the
// frame edge; a tap outside is_inside_filter_region (X, Y = plane position of the first
// pixel, limX / limY = plane extent of the mi grid) is replaced by the centre pixel,
// which contributes nothing to the sum, the minimum or the maximum -- exactly the
// reference's skipped tap.
typedef short cd2 __attribute__((ext_vector_type(2)));
DEV uint32_t cd_bytes(const uint8_t* t, int p)  // t[p .. p + 3], any alignment of p
{
    const uint32_t* w = reinterpret_cast<const uint32_t*>(t + (p & ~3));
    return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(p & 3));
}
DEV cd2 cd_lo(uint32_t w) { return __builtin_bit_cast(cd2, __builtin_amdgcn_perm(0u, w, 0x0c010c00u)); }
DEV cd2 cd_hi(uint32_t w) { return __builtin_bit_cast(cd2, __builtin_amdgcn_perm(0u, w, 0x0c030c02u)); }
DEV uint32_t cd_join(cd2 a, cd2 b)
{
    return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, a), 0x06040200u);
}
template <bool check>
DEV uint32_t cdef_quad(const uint8_t* t, int p, const int16_t* off, int pri, int sec, int damping, int X, int Y,
    int ts, int limX, int limY)
{
    const uint32_t xw = *reinterpret_cast<const uint32_t*>(t + p);
    // both strengths 0: every constrained difference is 0, so the clamp to the taps' range
    // returns x itself
    if (!pri && !sec) return xw;
    const cd2 x[2] = {cd_lo(xw), cd_hi(xw)};
    cd2 sum[2] = {cd2{0, 0}, cd2{0, 0}}, mx[2] = {x[0], x[1]}, mn[2] = {x[0], x[1]};
    const short adjP = (short)imax(0, damping - floor_log2(imax(pri, 1)));
    const short adjS = (short)imax(0, damping - floor_log2(imax(sec, 1)));
    const short tap0 = (pri & 1) ? 3 : 4, tap1 = (pri & 1) ? 3 : 2;  // Cdef_Pri_Taps
#pragma unroll
    for (int s = 0; s < 3; s++)
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
            const int o = off[s * 2 + kk];
#pragma unroll
            for (int sg = 0; sg < 2; sg++) {
                const int oo = sg ? o : -o;
                const uint32_t qw = cd_bytes(t, p + oo);
                cd2 q[2] = {cd_lo(qw), cd_hi(qw)};
                if (check) {
                    const int dy = (oo + 2 * ts + 2) / ts - 2;  // |dx|, |dy| <= 2
                    const int dx = oo - dy * ts;
                    const int yy = Y + dy, xx = X + dx;
                    const bool rowIn = yy >= 0 && yy < limY;
                    q[0].x = (rowIn && xx >= 0 && xx < limX) ? q[0].x : x[0].x;
                    q[0].y = (rowIn && xx + 1 >= 0 && xx + 1 < limX) ? q[0].y : x[0].y;
                    q[1].x = (rowIn && xx + 2 >= 0 && xx + 2 < limX) ? q[1].x : x[1].x;
                    q[1].y = (rowIn && xx + 3 >= 0 && xx + 3 < limX) ? q[1].y : x[1].y;
                }
                const short thr = s == 0 ? (short)pri : (short)sec, adj = s == 0 ? adjP : adjS;
                const short w = s == 0 ? (kk ? tap1 : tap0) : (kk ? 1 : 2);  // Cdef_Sec_Taps = {2, 1}
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    // constrain (Cdef.cpp:111-118): sign(d) * min(|d|, max(0, thr - (|d| >> adj))),
                    // i.e. d clamped to [-v, v] with v = max(0, thr - (|d| >> adj)) (v <= |d| is
                    // not needed: the clamp leaves a smaller |d| as it is); 0 for thr 0, so a
                    // tap of strength 0 only widens the range (min / max: every tap counts,
                    // Cdef.cpp:177-190)
                    if (thr) {
                        const cd2 d = q[h] - x[h];
                        const cd2 ad = __builtin_elementwise_max(d, -d);
                        const cd2 v = __builtin_elementwise_max(cd2{thr, thr} - (ad >> cd2{adj, adj}), cd2{0, 0});
                        const cd2 c = __builtin_elementwise_min(__builtin_elementwise_max(d, -v), v);
                        sum[h] += cd2{w, w} * c;
                    }
                    mx[h] = __builtin_elementwise_max(q[h], mx[h]);
                    mn[h] = __builtin_elementwise_min(q[h], mn[h]);
                }
            }
        }
    cd2 r[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        r[h] = x[h] + ((sum[h] + cd2{8, 8} + (sum[h] >> cd2{15, 15})) >> cd2{4, 4});  // (8 + sum - (sum < 0)) >> 4
        r[h] = __builtin_elementwise_min(__builtin_elementwise_max(r[h], mn[h]), mx[h]);
    }
    return cd_join(r[0], r[1]);
}

// Stage rows [y0 - 2, y0 + rows + 2) x columns [x0 - 4, x0 + cols + 4) of plane P into the
// tile t (row stride ts): aligned dwords where no coordinate needs clamping, else bytes
// with the coordinates clamped into the mi grid (taps beyond it are never used).
DEV void cd_stage(uint8_t* t, int ts, int nrows, const DevPlane& P, int x0, int y0, bool clamp, int mx, int my)
{
    const int ndw = ts / 4;
    if (!clamp) {
        for (int q = threadIdx.x; q < nrows * ndw; q += 256) {
            const int i = q / ndw, d = q - i * ndw;
            *reinterpret_cast<uint32_t*>(t + i * ts + 4 * d) =
                *reinterpret_cast<const uint32_t*>(P.p + (size_t)(y0 - CD_H + i) * P.stride + x0 - CD_X + 4 * d);
        }
        return;
    }
    for (int q = threadIdx.x; q < nrows * ts; q += 256) {
        const int i = q / ts, j = q - i * ts;
        t[i * ts + j] = px(P, CLIP3(0, mx, x0 - CD_X + j), CLIP3(0, my, y0 - CD_H + i));
    }
}

// grid (ceil(MiCols / 16), ceil(MiRows / 16), frames); reads k.dbk, writes k.cdef
DEV void cdef_body(const KParams* kps)
{
    __shared__ CdefLds L;
    const uint3 wg = xcd_block();  // (as lf_body)
    const KParams& k = KP(kps, wg.z);
    const int t = threadIdx.x;
    const int r0 = wg.y * 16, c0 = wg.x * 16;  // mi units
    if (r0 >= k.mi_rows || c0 >= k.mi_cols) return;
    const av1r_frame_hdr& h = *k.hdr;
    const int idx = k.cdef_idx[(r0 >> 4) * h.cdef_cols + (c0 >> 4)];
    const int rows4 = imin(16, k.mi_rows - r0), cols4 = imin(16, k.mi_cols - c0);
    const int x0 = c0 * 4, y0 = r0 * 4;
    if (idx == -1) {
        // not filtered: the output is the input (the reference filters into a copy), luma as
        // dwords (cols4 * 4 is a multiple of 4), chroma as 16-bit pairs (cols4 * 2 is even)
        const int nl = cols4, nc = cols4;  // dwords per luma row, 16-bit pairs per chroma row
        for (int q = t; q < rows4 * 4 * nl; q += 256) {
            const int i = q / nl, j = 4 * (q - i * nl);
            *reinterpret_cast<uint32_t*>(&px(k.cdef.pl[0], x0 + j, y0 + i)) = *reinterpret_cast<const uint32_t*>(&px(k.dbk.pl[0], x0 + j, y0 + i));
        }
        for (int q = t; q < 2 * rows4 * 2 * nc; q += 256) {
            const int pl = 1 + (q >= rows4 * 2 * nc), e = q - (pl - 1) * rows4 * 2 * nc;
            const int i = e / nc, j = 2 * (e - i * nc);
            *reinterpret_cast<uint16_t*>(&px(k.cdef.pl[pl], x0 / 2 + j, y0 / 2 + i)) =
                *reinterpret_cast<const uint16_t*>(&px(k.dbk.pl[pl], x0 / 2 + j, y0 / 2 + i));
        }
        return;
    }
    // cdef_block's skip test (Cdef.cpp:79-82) per 8x8 block, its mode-info loads issued with
    // the pixel loads below (one memory round trip for both)
    int fBlk = 0;
    if (t < 64) {
        const int br = r0 + (t >> 3) * 2, bc = c0 + (t & 7) * 2;
        if ((t >> 3) * 2 < rows4 && (t & 7) * 2 < cols4)
            fBlk = !((mi_at(k, br, bc).flags & AV1R_MI_SKIP) && (mi_at(k, br + 1, bc).flags & AV1R_MI_SKIP)
                && (mi_at(k, br, bc + 1).flags & AV1R_MI_SKIP) && (mi_at(k, br + 1, bc + 1).flags & AV1R_MI_SKIP));
    }
    const int limX = k.mi_cols * 4, limY = k.mi_rows * 4;
    const bool edge = x0 < CD_H || y0 < CD_H || x0 + 64 + CD_H > limX || y0 + 64 + CD_H > limY;
    const int cx0 = x0 / 2, cy0 = y0 / 2, climX = k.mi_cols * 2, climY = k.mi_rows * 2;
    const bool cedge = cx0 < CD_H || cy0 < CD_H || cx0 + 32 + CD_H > climX || cy0 + 32 + CD_H > climY;
    if (!edge && !cedge) {
        // away from the frame edges: every lane's dwords of the three tiles are loaded before
        // its first LDS store (one memory round trip; the staging loop waited once per
        // iteration, ~11 round trips per region)
        constexpr int NDY = CD_LS / 4, NY = CD_LR * NDY, QY = (NY + 255) / 256;
        constexpr int NDC = CD_CS / 4, NC = CD_CR * NDC, QC = (NC + 255) / 256;
        uint32_t vy[QY], vc[2][QC];
        // (lanes past a tile load its last dword again: no branch around the loads)
        const DevPlane PY = k.dbk.pl[0], PU = k.dbk.pl[1], PV = k.dbk.pl[2];
#pragma unroll
        for (int u = 0; u < QY; u++) {
            const int q = imin(t + 256 * u, NY - 1), i = q / NDY, d = q - i * NDY;
            vy[u] = *reinterpret_cast<const uint32_t*>(PY.p + (size_t)(y0 - CD_H + i) * PY.stride + x0 - CD_X + 4 * d);
        }
#pragma unroll
        for (int u = 0; u < QC; u++) {
            const int q = imin(t + 256 * u, NC - 1), i = q / NDC, d = q - i * NDC;
            const size_t o = (size_t)(cy0 - CD_H + i) * PU.stride + cx0 - CD_X + 4 * d;
            vc[0][u] = *reinterpret_cast<const uint32_t*>(PU.p + o);
            vc[1][u] = *reinterpret_cast<const uint32_t*>(PV.p + o);
        }
#pragma unroll
        for (int u = 0; u < QY; u++) {
            const int q = t + 256 * u, i = q / NDY, d = q - i * NDY;
            if (q < NY) *reinterpret_cast<uint32_t*>(&L.y[i][4 * d]) = vy[u];
        }
#pragma unroll
        for (int pl = 0; pl < 2; pl++)
#pragma unroll
            for (int u = 0; u < QC; u++) {
                const int q = t + 256 * u, i = q / NDC, d = q - i * NDC;
                if (q < NC) *reinterpret_cast<uint32_t*>(&L.uv[pl][i][4 * d]) = vc[pl][u];
            }
    } else {
        cd_stage(&L.y[0][0], CD_LS, CD_LR, k.dbk.pl[0], x0, y0, edge, limX - 1, limY - 1);
        cd_stage(&L.uv[0][0][0], CD_CS, CD_CR, k.dbk.pl[1], cx0, cy0, cedge, climX - 1, climY - 1);
        cd_stage(&L.uv[1][0][0], CD_CS, CD_CR, k.dbk.pl[2], cx0, cy0, cedge, climX - 1, climY - 1);
    }
    if (t < 64) L.filt[t] = (uint8_t)fBlk;
    __syncthreads();
    // direction costs: wave w (wave-uniform directions 2w and 2w + 1), lane = 8x8 block; the
    // block's 64 pixels read once as 16 dwords and kept in registers for both directions
    {
        const int b = t & 63, w = t >> 6;
        if (L.filt[b]) {
            const int bx = (b & 7) * 8, by = (b >> 3) * 8;
            // rows in the order i ^ 4 for block rows 2, 3, 6, 7 (banks: header above)
            const int rot = (b >> 4) & 1;
            // (each row index opaque to the compiler: one ds_read_b64 per row, not pairs
            // merged into ds_read2_b64, whose 16-lane groups bank mod 32)
            uint64_t v[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                int row = CD_H + by + (i ^ (4 * rot));
                asm volatile("" : "+v"(row));
                v[i] = *reinterpret_cast<const uint64_t*>(&L.y[row][CD_X + bx]);
            }
            uint32_t rw[8][2];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const uint64_t r = rot ? v[i ^ 4] : v[i];
                rw[i][0] = (uint32_t)r;
                rw[i][1] = (uint32_t)(r >> 32);
            }
            auto px8 = [&](int i, int j) { return (int)((rw[i][j >> 2] >> (8 * (j & 3))) & 0xff) - 128; };
            int c0, c1;
            switch (__builtin_amdgcn_readfirstlane(w)) {
            case 0: c0 = cdef_cost_f<0>(px8), c1 = cdef_cost_f<1>(px8); break;
            case 1: c0 = cdef_cost_f<2>(px8), c1 = cdef_cost_f<3>(px8); break;
            case 2: c0 = cdef_cost_f<4>(px8), c1 = cdef_cost_f<5>(px8); break;
            default: c0 = cdef_cost_f<6>(px8), c1 = cdef_cost_f<7>(px8); break;
            }
            L.cost[b][2 * w] = c0;
            L.cost[b][2 * w + 1] = c1;
        }
    }
    __syncthreads();
    if (t < 64 && L.filt[t]) {
        int best = 0, yDir = 0;
        for (int d = 0; d < 8; d++)
            if (L.cost[t][d] > best) {
                best = L.cost[t][d];
                yDir = d;
            }
        const int var = (best - L.cost[t][(yDir + 4) & 7]) >> 10;
        int priStr = h.cdef_y_pri[idx];
        const int varStr = (var >> 6) ? imin(floor_log2(var >> 6), 12) : 0;
        L.pri[t] = (int16_t)(var ? (priStr * (4 + varStr) + 8) >> 4 : 0);
        // tap offsets: luma direction (0 when the primary strength is 0), chroma direction
        // Cdef_Uv_Dir (identity for 4:2:0; 0 when the chroma primary strength is 0)
        const int dy0 = priStr == 0 ? 0 : yDir, dc0 = h.cdef_uv_pri[idx] == 0 ? 0 : av1r_cdef_uv_dir420[yDir];
#pragma unroll
        for (int s = 0; s < 3; s++)
#pragma unroll
            for (int kk = 0; kk < 2; kk++) {
                const int dl = s == 0 ? dy0 : ((dy0 + (s == 1 ? -2 : 2)) & 7);
                const int dc = s == 0 ? dc0 : ((dc0 + (s == 1 ? -2 : 2)) & 7);
                L.offY[t][s * 2 + kk] = (int16_t)(av1r_cdef_directions[dl][kk][0] * CD_LS + av1r_cdef_directions[dl][kk][1]);
                L.offC[t][s * 2 + kk] = (int16_t)(av1r_cdef_directions[dc][kk][0] * CD_CS + av1r_cdef_directions[dc][kk][1]);
            }
    }
    __syncthreads();
    // luma: half-wave hw = block row; lane (k, d) takes the 4-pixel group d (0..15) of rows
    // u + 4k (u = 0..3) of that block row, all in the 8x8 block d / 2
    {
        const int bi = t >> 5, d = t & 15, kq = (t >> 4) & 1;
        const int b = bi * 8 + (d >> 1);
        const int j0 = 4 * d;
        const int ySec = h.cdef_y_sec[idx];
        if (d < cols4) {  // (a group is one mi column)
            const bool f = L.filt[b];
            const int pri = L.pri[b];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = bi * 8 + u + 4 * kq;
                if (i >= rows4 * 4) break;
                const int p = (CD_H + i) * CD_LS + CD_X + j0;
                uint32_t o;
                if (!f) o = *reinterpret_cast<const uint32_t*>(&L.y[0][0] + p);
                else if (edge)
                    o = cdef_quad<true>(&L.y[0][0], p, L.offY[b], pri, ySec, h.cdef_damping, x0 + j0, y0 + i, CD_LS, limX, limY);
                else
                    o = cdef_quad<false>(&L.y[0][0], p, L.offY[b], pri, ySec, h.cdef_damping, 0, 0, CD_LS, 0, 0);
                *reinterpret_cast<uint32_t*>(&px(k.cdef.pl[0], x0 + j0, y0 + i)) = o;
            }
        }
    }
    // chroma: half-wave hw -> plane hw / 4 and 8 rows (two 4x4 block rows); lane (k, d) takes
    // the 4-pixel group d (one 4x4 block column) of rows u + 2k (u = 0, 1), in block row k / 2
    {
        const int uvPri = h.cdef_uv_pri[idx], uvSec = h.cdef_uv_sec[idx];
        const int hw = t >> 5, pl = hw >> 2, bj = t & 7, kq = (t >> 3) & 3;
        const int bi = 2 * (hw & 3) + (kq >> 1), b = bi * 8 + bj;
        const int j0 = bj * 4;
        if (j0 < cols4 * 2) {
            const bool full = j0 + 4 <= cols4 * 2;  // else only the left 2 columns are in the grid
            const bool f = L.filt[b];
            const uint8_t* tile = &L.uv[pl][0][0];
#pragma unroll
            for (int r = 0; r < 2; r++) {
                const int i = 8 * (hw & 3) + r + 2 * kq;
                if (i >= rows4 * 2) break;
                const int p = (CD_H + i) * CD_CS + CD_X + j0;
                uint32_t o;
                if (!f) o = *reinterpret_cast<const uint32_t*>(tile + p);
                else if (cedge)
                    o = cdef_quad<true>(tile, p, L.offC[b], uvPri, uvSec, h.cdef_damping - 1, cx0 + j0, cy0 + i, CD_CS, climX, climY);
                else
                    o = cdef_quad<false>(tile, p, L.offC[b], uvPri, uvSec, h.cdef_damping - 1, 0, 0, CD_CS, 0, 0);
                uint8_t* dst = &px(k.cdef.pl[1 + pl], cx0 + j0, cy0 + i);
                if (full) *reinterpret_cast<uint32_t*>(dst) = o;
                else *reinterpret_cast<uint16_t*>(dst) = (uint16_t)o;
            }
        }
    }
}
// (6 waves per SIMD instead of 5 measured no faster: the filters are not occupancy-bound)
extern "C" __global__ __launch_bounds__(256) void k_cdef(const KParams* kps) { cdef_body(kps); }

// ------------------------------------------------------------------------------------
// Loop restoration
// ------------------------------------------------------------------------------------
struct LrPix {
    DevPlane cdefP;  // CDEF output (k.cdef)
    DevPlane preP;   // deblocked, pre-CDEF frame (k.dbk)
    int start, end;  // stripe
};
// get_source_sample (LoopRestoration.cpp:234-246) + extendBorder(3) as clamping
DEV int lr_src(const LrPix& S, int x, int y)
{
    const bool pre = y < S.start || y >= S.end;
    if (y < S.start) y = imax(S.start - 2, y);
    else if (y >= S.end) y = imin(S.end + 1, y);
    const uint8_t* base = pre ? S.preP.p : S.cdefP.p;  // (selects values: no struct address)
    const int stride = pre ? S.preP.stride : S.cdefP.stride;
    x = CLIP3(0, S.cdefP.w - 1, x);
    y = CLIP3(0, S.cdefP.h - 1, y);
    return base[(size_t)y * stride + x];
}

// Four values in 0..255 as the bytes of a dword, through v_perm: written as shifts and ORs,
// hipcc (ROCm 7.2) folds the clamp, shift and byte packing of two of them into
// v_ashr_pk_u8_i32, which on gfx950 leaves the destination's upper half as it was while the
// compiler assumes it zero -- bytes 2 of the packed dword came out ORed with stale bits
// (measured: the loop-restoration output wrong at every x % 4 == 2 pixel).
DEV uint32_t pack_u8x4(int a, int b, int c, int d)
{
    const uint32_t lo = __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x0c0c0400u);  // {a, b, 0, 0}
    const uint32_t hi = __builtin_amdgcn_perm((uint32_t)d, (uint32_t)c, 0x0c0c0400u);  // {c, d, 0, 0}
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// Tiles of LR_TW columns x one half-stripe (luma) / one stripe (chroma) rows: inside a
// tile the stripe (hence get_source_sample's row mapping) and the restoration-unit row are
// fixed, so the source is staged once in LDS with its 3-pixel halo and every filter reads
// only LDS.  Restoration units are at least 32 wide: a tile meets at most 3 unit columns.
#define LR_TW 64
#define LR_TH 32
#define LR_SW (LR_TW + 8)
// The Wiener intermediates and the self-guided a/b planes share their LDS: a tile whose
// units mix both types is filtered in two rounds (Wiener, then self-guided).  29.7 KB:
// 5 workgroups per CU (34.5 KB and 4 without the union)
struct LrLds {
    uint8_t src[LR_TH + 6][LR_SW];            // get_source_sample over rows ty0-3.., cols x0-4..
    union {
        int16_t hw[LR_TH + 6][LR_TW];         // Wiener horizontal pass
        struct {
            int16_t A[2][LR_TH + 2][LR_TW + 2];  // self-guided a per pass, rows ty0-1.., cols x0-1..
            int32_t B[2][LR_TH + 2][LR_TW + 2];
        };
    };
    av1r_lr_unit unit[3];
};

// Per-set constants of the self-guided filter, folded at compile time: s = the box
// scale of LoopRestoration.cpp:370 (((1 << 20) + n^2 eps / 2) / (n^2 eps), n = 25 / 9 for
// r = 2 / 1) and the divisions ((z << 8) + z / 2) / (z + 1) of :374-378 for z in 0..255.
struct SgrTabs {
    uint32_t s[16][2];
    uint16_t xbyx1[256];
};
constexpr SgrTabs make_sgr_tabs()
{
    SgrTabs t{};
    const int prm[16][4] = {{2, 12, 1, 4}, {2, 15, 1, 6}, {2, 18, 1, 8}, {2, 21, 1, 9}, {2, 24, 1, 10}, {2, 29, 1, 11},
        {2, 36, 1, 12}, {2, 45, 1, 13}, {2, 56, 1, 14}, {2, 68, 1, 15}, {0, 0, 1, 5}, {0, 0, 1, 8}, {0, 0, 1, 11},
        {0, 0, 1, 14}, {2, 30, 0, 0}, {2, 75, 0, 0}};  // Sgr_Params (Av1Common.h:206-211)
    for (int set = 0; set < 16; set++)
        for (int pass = 0; pass < 2; pass++) {
            const int r = prm[set][pass * 2], eps = prm[set][pass * 2 + 1];
            const int n = (2 * r + 1) * (2 * r + 1), n2e = n * n * eps;
            t.s[set][pass] = r ? (uint32_t)(((1 << 20) + n2e / 2) / n2e) : 0u;
        }
    t.xbyx1[0] = 1;
    for (int z = 1; z < 255; z++) t.xbyx1[z] = (uint16_t)(((z << 8) + (z / 2)) / (z + 1));
    t.xbyx1[255] = 256;
    return t;
}
__constant__ SgrTabs g_sgr = make_sgr_tabs();

// a, b of the self-guided box at staged position (si, sj) = source (row, col) index of the
// box centre (LoopRestoration.cpp:284-380, restated per position; 32-bit arithmetic as
// the reference's)
DEV void sgr_ab_fin(int a, int b, int r, int set, int pass, int& A, int& B)
{
    const int n = r == 2 ? 25 : 9;  // (2r + 1)^2 (r is 1 or 2)
    const uint32_t s = g_sgr.s[set][pass];
    int p = imax(0, a * n - b * b);
    int z = (int)((uint32_t)p * s + (1u << 19)) >> 20;
    int a2;
    if (z >= 0) a2 = g_sgr.xbyx1[imin(z, 255)];
    else a2 = ((z << 8) + (z / 2)) / (z + 1);  // the 32-bit wrap-around case, as the reference
    const int oneOverN = r == 2 ? 164 : 455;  // ((1 << 12) + n / 2) / n
    int b2 = ((1 << 8) - a2) * b * oneOverN;
    A = a2;
    B = r2(b2, 12);
}
DEV void sgr_ab_lds(const LrLds& L, int si, int sj, int r, int set, int pass, int& A, int& B)
{
    int a = 0, b = 0;
    for (int dy = -r; dy <= r; dy++)
        for (int dx = -r; dx <= r; dx++) {
            int cv = L.src[si + dy][sj + dx];
            a += cv * cv;
            b += cv;
        }
    sgr_ab_fin(a, b, r, set, pass, A, B);
}

// LoopRestoration's filters over one staged tile (L.src, L.unit ready; the caller's
// barrier after staging): Wiener (LoopRestoration.cpp:247-277) and self-guided (:284-479),
// rows [ty0, ty0 + th) x columns [x0, x0 + tw) of plane `plane`, written to O.  y0: the
// stripe's first row (forEachBlock's y); us / cols / uc0 / nU: unit size, unit columns of the
// plane, the tile's first unit column and its unit count.
DEV void lr_filter_tile(LrLds& L, const av1r_frame_hdr& h, int plane, int x0, int tw, int ty0, int th, int y0, int us,
    int cols, int uc0, int nU, int planeEndX, int planeEndY, const DevPlane& O)
{
    const int t = threadIdx.x;
    int anyW = 0, anyS = 0;
    for (int u = 0; u < nU; u++) {
        anyW |= L.unit[u].type == AV1R_RESTORE_WIENER;
        anyS |= L.unit[u].type == AV1R_RESTORE_SGRPROJ;
    }
    const int usl = __builtin_ctz((unsigned)us);  // unit sizes are powers of two (32..256, validate())
    auto unitOf = [&](int c) { return imin((x0 + CLIP3(0, tw - 1, c)) >> usl, cols - 1) - uc0; };
    // q -> (row, column) of a tw-wide tile: a shift for the full-width tiles
    const bool fullW = tw == LR_TW;
    const int rounds = anyW && anyS ? 2 : 1;
    for (int rd = 0; rd < rounds; rd++) {
        const bool doW = anyW && (rounds == 1 || rd == 0), doS = anyS && (rounds == 1 || rd == 1);
        if (rd) __syncthreads();  // round 0's reads of the shared LDS are done
        if (doW) {
            // wienerFilter horizontal pass (LoopRestoration.cpp:253-265), four columns per lane:
            // a 4-column group lies in one restoration unit (units start at multiples of 32 of
            // the plane, x0 at a multiple of 64), its 10 source bytes come from 3 aligned dwords
            const int offset = 1 << (8 + 7 - 3 - 1), limit = (1 << (8 + 1 + 7 - 3)) - 1;
            const int ng = (tw + 3) >> 2;
            for (int q = t; q < (th + 6) * ng; q += 256) {
                const int i = fullW ? q >> 4 : q / ng, c0 = 4 * (q - i * ng);
                const av1r_lr_unit& u = L.unit[unitOf(c0)];
                if (u.type != AV1R_RESTORE_WIENER) continue;
                const int f0 = u.wiener[1][0], f1 = u.wiener[1][1], f2 = u.wiener[1][2];
                const int hf3 = 128 - 2 * (f0 + f1 + f2);
                const uint32_t* w = reinterpret_cast<const uint32_t*>(&L.src[i][c0]);
                const uint32_t d0 = w[0], d1 = w[1], d2 = w[2];
                int sp[10];  // L.src[i][c0 + 1 + k]
#pragma unroll
                for (int k = 0; k < 10; k++) {
                    const int b = k + 1;
                    const uint32_t dw = b < 4 ? d0 : (b < 8 ? d1 : d2);
                    sp[k] = (dw >> (8 * (b & 3))) & 0xff;
                }
                int o[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int hs = f0 * (sp[j] + sp[j + 6]) + f1 * (sp[j + 1] + sp[j + 5]) + f2 * (sp[j + 2] + sp[j + 4]) + hf3 * sp[j + 3];
                    o[j] = CLIP3(-offset, limit - offset, r2(hs, 3)) & 0xffff;
                }
                *reinterpret_cast<uint2*>(&L.hw[i][c0]) = make_uint2((uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16));
            }
        }
        if (doS) {
            // a, b of both passes (box radius 2 / 1: Sgr_Params) at rows ty0-1 .. ty1 (ii), cols
            // x0-1 .. x0+tw (cc).  The box sums are separable: each lane walks one column over a
            // run of rows, keeping the last five rows' horizontal 5- and 3-sums in registers.
            constexpr int RUNS = 3;
            const int nr = th + 2, nc = tw + 2, runH = (nr + RUNS - 1) / RUNS;
            for (int q = t; q < RUNS * nc; q += 256) {
                const int cc = q % nc, i0 = (q / nc) * runH, i1 = imin(nr, i0 + runH);
                const av1r_lr_unit& u = L.unit[unitOf(cc - 1)];
                if (u.type != AV1R_RESTORE_SGRPROJ || i0 >= i1) continue;
                const int set = u.sgr_set;
                const bool p0 = av1r_sgr_params[set][0] != 0, p1 = av1r_sgr_params[set][2] != 0;
                // h5[k] / h3[k]: (squares, sums) of source row sr - k, columns cc+1..cc+5 / cc+2..cc+4
                int a5[5] = {}, b5[5] = {}, a3[4] = {}, b3[4] = {};
                for (int sr = i0; sr < i1 + 4; sr++) {
    #pragma unroll
                    for (int k = 4; k > 0; k--) {
                        a5[k] = a5[k - 1];
                        b5[k] = b5[k - 1];
                    }
    #pragma unroll
                    for (int k = 3; k > 0; k--) {
                        a3[k] = a3[k - 1];
                        b3[k] = b3[k - 1];
                    }
                    const uint8_t* row = &L.src[sr][cc + 1];
                    const int v0 = row[0], v1 = row[1], v2 = row[2], v3 = row[3], v4 = row[4];
                    b3[0] = v1 + v2 + v3;
                    a3[0] = v1 * v1 + v2 * v2 + v3 * v3;
                    b5[0] = b3[0] + v0 + v4;
                    a5[0] = a3[0] + v0 * v0 + v4 * v4;
                    const int ii = sr - 4;  // the box centre's row: source row ii + 2
                    if (ii < i0) continue;
                    int A, B;
                    if (p0 && ((ty0 - 1 + ii - y0) & 1)) {  // pass 0 uses odd rows only
                        sgr_ab_fin(a5[0] + a5[1] + a5[2] + a5[3] + a5[4], b5[0] + b5[1] + b5[2] + b5[3] + b5[4], 2, set, 0, A, B);
                        L.A[0][ii][cc] = (int16_t)A;
                        L.B[0][ii][cc] = B;
                    }
                    if (p1) {  // rows ii + 1 .. ii + 3
                        sgr_ab_fin(a3[1] + a3[2] + a3[3], b3[1] + b3[2] + b3[3], 1, set, 1, A, B);
                        L.A[1][ii][cc] = (int16_t)A;
                        L.B[1][ii][cc] = B;
                    }
                }
            }
        }
        __syncthreads();
        // the output, four pixels per lane (one dword store): the group's unit and its
        // parameters once, the Wiener column sums from int16 pairs, the self-guided A / B of
        // the six columns c0 - 1 .. c0 + 4 once per row and pass, their cross-unit columns (only
        // a group at a unit boundary has one) recomputed with this unit's set
        const int ng = (tw + 3) >> 2;
        for (int q = t; q < ng * th; q += 256) {
            const int r = fullW ? q >> 4 : q / ng, c0 = 4 * (q - r * ng);
            const int x = x0 + c0, y = ty0 + r;
            const uint32_t cw = *reinterpret_cast<const uint32_t*>(&L.src[r + 3][c0 + 4]);
            const int ui = unitOf(c0);
            const av1r_lr_unit& u = L.unit[ui];
            // (x < planeEndX, y < planeEndY hold for every pixel of the tile: tw, th stop at the
            // plane's edge, which is planeEndX / planeEndY)
            const bool filt = u.type != AV1R_RESTORE_NONE;
            // this round's groups: Wiener and unfiltered ones in round 0, self-guided in round 1
            if (rounds == 2 && (rd == 1) != (filt && u.type == AV1R_RESTORE_SGRPROJ)) continue;
            uint32_t ow = cw;
            if (filt && u.type == AV1R_RESTORE_WIENER) {
                const int g0 = u.wiener[0][0], g1 = u.wiener[0][1], g2 = u.wiener[0][2];
                const int vf3 = 128 - 2 * (g0 + g1 + g2);
                int hv[7][4];
#pragma unroll
                for (int k = 0; k < 7; k++)
#pragma unroll
                    for (int j = 0; j < 4; j++) hv[k][j] = L.hw[r + k][c0 + j];
                int o[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int sum = g0 * (hv[0][j] + hv[6][j]) + g1 * (hv[1][j] + hv[5][j]) + g2 * (hv[2][j] + hv[4][j]) + vf3 * hv[3][j];
                    o[j] = clip1(r2(sum, 11));
                }
                ow = pack_u8x4(o[0], o[1], o[2], o[3]);
            } else if (filt) {
                // selfGuidedFilter (LoopRestoration.cpp:420-479)
                const int set = u.sgr_set;
                const int i = y - y0;
                const int w0 = u.sgr_xqd[0], w1 = u.sgr_xqd[1], w2 = (1 << 7) - w0 - w1;
                const bool crossL = c0 > 0 && unitOf(c0 - 1) != ui, crossR = unitOf(c0 + 4) != ui;
                int px4[4], v[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    px4[j] = (cw >> (8 * j)) & 0xff;
                    v[j] = w1 * (px4[j] << 4);
                }
#pragma unroll
                for (int pass = 0; pass < 2; pass++) {
                    const int rad = av1r_sgr_params[set][pass * 2];
                    const int w = pass ? w2 : w0;
                    if (!rad) {
#pragma unroll
                        for (int j = 0; j < 4; j++) v[j] += w * (px4[j] << 4);
                        continue;
                    }
                    const int shift = (pass == 0 && (i & 1)) ? 4 : 5;
                    int a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int dy = -1; dy <= 1; dy++) {
                        if (pass == 0 && !((i + dy) & 1)) continue;
                        // A / B of columns c0 - 1 .. c0 + 4 (indices c0 .. c0 + 5 of the a/b planes)
                        int Av[6], Bv[6];
                        const uint32_t* ap = reinterpret_cast<const uint32_t*>(&L.A[pass][r + 1 + dy][c0]);
#pragma unroll
                        for (int k = 0; k < 3; k++) {
                            const uint32_t d = ap[k];
                            Av[2 * k] = (int16_t)(d & 0xffff);
                            Av[2 * k + 1] = (int16_t)(d >> 16);
                        }
#pragma unroll
                        for (int k = 0; k < 6; k++) Bv[k] = L.B[pass][r + 1 + dy][c0 + k];
                        if (crossL) sgr_ab_lds(L, r + 3 + dy, c0 + 3, rad, set, pass, Av[0], Bv[0]);
                        if (crossR) sgr_ab_lds(L, r + 3 + dy, c0 + 8, rad, set, pass, Av[5], Bv[5]);
#pragma unroll
                        for (int j = 0; j < 4; j++)
#pragma unroll
                            for (int dx = -1; dx <= 1; dx++) {
                                const int wt = pass == 0 ? (dx == 0 ? 6 : 5) : ((dx == 0 || dy == 0) ? 4 : 3);
                                a[j] += wt * Av[j + 1 + dx];
                                b[j] += wt * Bv[j + 1 + dx];
                            }
                    }
#pragma unroll
                    for (int j = 0; j < 4; j++) v[j] += w * r2(a[j] * px4[j] + b[j], 8 + shift - 4);
                }
                ow = pack_u8x4(clip1(r2(v[0], 4 + 7)), clip1(r2(v[1], 4 + 7)), clip1(r2(v[2], 4 + 7)), clip1(r2(v[3], 4 + 7)));
            }
            uint8_t* dst = O.p + (size_t)y * O.stride + x;
            if (c0 + 4 <= tw) *reinterpret_cast<uint32_t*>(dst) = ow;
            else
                for (int j = 0; j < tw - c0; j++) dst[j] = (uint8_t)(ow >> (8 * j));
        }
    }
}

// one 256-lane workgroup per tile; wg = (64-column tile, tile row, 3 * frame + plane).  Reads
// the CDEF frame (k.cdef) and the deblocked frame (k.dbk, stripe rows), writes k.lrout.
// What a launch must guarantee: every tile of every frame and plane is
// some workgroup's wg, and a tile row is a LUMA half-stripe (two per 64-row stripe from -8)
// but a whole CHROMA stripe (one per 32-row stripe from -4) -- wg.y means a different row
// span per plane (the static_assert below).  Nothing else of the launch enters: a workgroup
// reads only its own tile's inputs, so any order, grid shape or residency gives the same
// output.  Round 6 re-created round 5's "one-grid" variant (k_lr1 below, every frame's luma
// then chroma tiles in a 1-D grid): 172 streams stage-exact plus the synthetic tests
// (profiles/r06_lr_onegrid_parity.txt), so its round-5 mismatch was that variant's own tile
// numbering, not a property of this kernel.  The one-grid form is also the faster (LR 0.0125
// -> 0.0121 ms per 1080p frame, profiles/r06_ab_lr_onegrid.txt) and is k_lr since.
static_assert(64 / LR_TH == 2 && 32 / LR_TH == 1, "k_lr tile rows: luma half-stripes, chroma whole stripes");
DEV void lr_body(const KParams* kps, const uint3 wg)
{
    __shared__ LrLds L;
    const int t = threadIdx.x;
    const KParams& k = KP(kps, wg.z / 3);
    if (!k.hdr->uses_lr) return;  // the frame's output is its CDEF frame
    const int plane = wg.z % 3, sub = plane ? 1 : 0;
    const DevPlane C = k.cdef.pl[plane];
    const DevPlane O = k.lrout.pl[plane];
    const int x0 = wg.x * LR_TW;
    if (x0 >= C.w) return;
    const int stripeH = 64 >> sub, off = 8 >> sub;
    const int perStripe = stripeH / LR_TH;
    const int sNum = wg.y / perStripe, half = wg.y - sNum * perStripe;
    LrPix S;
    S.cdefP = C;
    S.preP = k.dbk.pl[plane];
    S.start = sNum * stripeH - off;
    S.end = S.start + stripeH;
    const int ty0 = imax(0, S.start + half * LR_TH), ty1 = imin(S.start + (half + 1) * LR_TH, C.h);
    if (ty0 >= ty1) return;
    const int tw = imin(LR_TW, C.w - x0), th = ty1 - ty0;
    const av1r_frame_hdr& h = *k.hdr;
    if (h.lr_type[plane] == AV1R_RESTORE_NONE) {
        // the CDEF frame copied: a dword per lane (x0 a multiple of 64, strides of 256), the
        // plane's last 1-3 columns (odd chroma widths) by bytes
        const int ng = (tw + 3) >> 2;
        for (int q = t; q < ng * th; q += 256) {
            const int r = q / ng, c = 4 * (q - r * ng);
            const uint8_t* sp = C.p + (size_t)(ty0 + r) * C.stride + x0 + c;
            uint8_t* dp = O.p + (size_t)(ty0 + r) * O.stride + x0 + c;
            if (c + 4 <= tw) *reinterpret_cast<uint32_t*>(dp) = *reinterpret_cast<const uint32_t*>(sp);
            else
                for (int j = 0; j < tw - c; j++) dp[j] = sp[j];
        }
        return;
    }
    const int us = h.lr_unit_size[plane];
    const int rows = h.lr_unit_rows[plane], cols = h.lr_unit_cols[plane];
    const int planeEndX = r2(k.frame_w, sub), planeEndY = r2(k.frame_h, sub);
    const int ur = imin((ty0 + off) / us, rows - 1);  // one unit row per stripe
    const int uc0 = imin(x0 / us, cols - 1);
    const int nU = imin((x0 + tw - 1) / us, cols - 1) - uc0 + 1;
    if (t < nU) L.unit[t] = k.lr[h.lr_unit_off[plane] + ur * cols + uc0 + t];
    const int y0 = imax(S.start, 0);  // forEachBlock's y: the stripe's first row
    // stage the source rows ty0-3 .. ty1+2, cols x0-4 .. x0+67 (L.src[i][j]: x = x0 - 4 + j):
    // aligned dwords where no column needs clamping, else bytes; every lane's loads are
    // issued before its LDS stores
    if (x0 >= 4 && x0 + LR_SW - 4 <= C.w) {
        constexpr int ND = LR_SW / 4, NQ = ((LR_TH + 6) * ND + 255) / 256;
        uint32_t v[NQ];
#pragma unroll
        for (int u = 0; u < NQ; u++) {
            const int q = t + 256 * u, i = q / ND, d = q - i * ND;
            if (i < th + 6) {
                int y = ty0 - 3 + i;  // get_source_sample's row mapping
                const bool pre = y < S.start || y >= S.end;
                if (y < S.start) y = imax(S.start - 2, y);
                else if (y >= S.end) y = imin(S.end + 1, y);
                y = CLIP3(0, C.h - 1, y);
                const uint8_t* row = (pre ? S.preP.p : C.p) + (size_t)y * (pre ? S.preP.stride : C.stride);
                v[u] = *reinterpret_cast<const uint32_t*>(row + x0 - 4 + 4 * d);
            }
        }
#pragma unroll
        for (int u = 0; u < NQ; u++) {
            const int q = t + 256 * u, i = q / ND, d = q - i * ND;
            if (i < th + 6) *reinterpret_cast<uint32_t*>(&L.src[i][4 * d]) = v[u];
        }
    } else {
        constexpr int NQ = ((LR_TH + 6) * LR_SW + 255) / 256;
        uint8_t v[NQ];
#pragma unroll
        for (int u = 0; u < NQ; u++) {
            const int q = t + 256 * u, i = q / LR_SW, j = q - i * LR_SW;
            if (i < th + 6) v[u] = (uint8_t)lr_src(S, x0 - 4 + j, ty0 - 3 + i);
        }
#pragma unroll
        for (int u = 0; u < NQ; u++) {
            const int q = t + 256 * u, i = q / LR_SW, j = q - i * LR_SW;
            if (i < th + 6) L.src[i][j] = v[u];
        }
    }
    __syncthreads();
    lr_filter_tile(L, h, plane, x0, tw, ty0, th, y0, us, cols, uc0, nU, planeEndX, planeEndY, O);
}
// Every frame's luma tiles (nxl x nyl) then its chroma tiles (nxc x nyc per plane) in one 1-D
// grid: no empty workgroups (round 5's 3-D grid sized every plane by the luma tiles, so three
// quarters of the chroma workgroups started and returned at once).  Dispatch order (round 4:
// XCD order for LR fetched 16.7 -> 6.7 MB/frame but took 4K LR 0.080 -> 0.108 ms/frame).
extern "C" __global__ __launch_bounds__(256) void k_lr(const KParams* kps, int nxl, int nyl, int nxc, int nyc)
{
    const int per = nxl * nyl + 2 * nxc * nyc;
    const int f = blockIdx.x / per;
    int r = blockIdx.x - f * per, plane = 0, nx = nxl;
    if (r >= nxl * nyl) {
        r -= nxl * nyl;
        plane = 1 + r / (nxc * nyc);
        r -= (plane - 1) * nxc * nyc;
        nx = nxc;
    }
    lr_body(kps, make_uint3(r % nx, r / nx, 3 * f + plane));
}

// The launch metadata, copied by the compute queue itself from pinned host memory (the
// device reads it over the bus, bypassing the caches): no copy-engine hand-off between a
// batch's last filter and the next batch's first kernel (an SDMA copy there started
// ~75 us after the preceding kernel ended).
extern "C" __global__ __launch_bounds__(256) void k_fetch(uint32_t* __restrict__ dst, uint32_t* src, size_t n4)
{
    // system-scope loads (sc0 sc1): never a stale cached copy of the host's rewritten ring slot
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
void launch_k_fetch(void* dst, const void* src, size_t bytes, hipStream_t s)
{
    const size_t n4 = (bytes + 3) / 4;
    const unsigned grid = (unsigned)std::min<size_t>(1024, (n4 + 255) / 256);
    hipLaunchKernelGGL(k_fetch, dim3(grid ? grid : 1), dim3(256), 0, s, reinterpret_cast<uint32_t*>(dst),
        reinterpret_cast<uint32_t*>(const_cast<void*>(src)), n4);
}

// ------------------------------------------------------------------------------------
// k_mi: the mode-info grid of each frame of the launch, derived from its records instead of
// uploaded (24 B per 4x4 unit: 3.1 MB of a 1080p frame's ~7.6 MB batch).  What the parser
// stores per 4x4 (Block::parse, Block.cpp:322-362) is the block's mode info over its units;
// LoopfilterTxSizes is the transform size over the units each transform block covers, the
// luma units under a chroma one included (TransformBlock::decode, TransformBlock.cpp:
// 2444-2454); units outside the frame that no block reaches stay zero.  Three launches (one
// frame per grid row): zero the out-of-frame units, write the blocks' units (16 lanes per
// block), then the transform blocks' lf_tx bytes.
// ------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(256) void k_mi_zero(const KParams* kps)
{
    const KParams& k = KP(kps, blockIdx.y);
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    // k_flow's done words start at 0, no launch's epoch (they are not uploaded); a tiny item's
    // slot gets its TinyItem (av1r_dev.h)
    if (i < k.n_items && k.done) {
        k.done[i] = 0;
        WorkItem* items = const_cast<WorkItem*>(k.items);
        const WorkItem w = items[i];
        if (w.hflags & AV1R_WI_TINY) {
            const TinyItem r = tiny_from_item(k, w, k.blocks[w.block], k.deps + w.dep_off - 4);
            *reinterpret_cast<TinyItem*>(items + i) = r;
        }
    }
    const int r = (int)(i / (uint32_t)k.mi_stride), c = (int)(i - (uint32_t)r * k.mi_stride);
    if (r >= k.mi_rows_alloc || (r < k.mi_rows && c < k.mi_cols)) return;
    uint32_t* d = reinterpret_cast<uint32_t*>(const_cast<av1r_mi*>(k.mi) + i);
#pragma unroll
    for (int w = 0; w < 6; w++) d[w] = 0;
}
extern "C" __global__ __launch_bounds__(256) void k_mi_blocks(const KParams* kps)
{
    const KParams& k = KP(kps, blockIdx.y);
    const uint32_t bi = blockIdx.x * 16 + (threadIdx.x >> 4);
    if (bi >= k.n_blocks) return;
    const DevBlock& b = k.blocks[bi];
    av1r_mi m;
    memset(&m, 0, sizeof(m));
    for (int l = 0; l < 2; l++) {
        m.mv[l][0] = b.mv[l][0];
        m.mv[l][1] = b.mv[l][1];
        m.ref_frame[l] = b.ref_frame[l];
    }
    m.mi_size = b.mi_size;
    m.y_mode = b.y_mode;
    m.filt = b.filt;
    m.flags = (uint8_t)(((b.flags & AV1R_BLK_SKIP) ? AV1R_MI_SKIP : 0) | ((b.flags & AV1R_BLK_INTER) ? AV1R_MI_INTER : 0));
    for (int i = 0; i < 4; i++) m.delta_lf[i] = b.delta_lf[i];
    m.uv_mode = b.uv_mode;
    uint32_t w[6];
    memcpy(w, &m, sizeof(w));
    const int bw4 = av1r_num4x4w[b.mi_size], bh4 = av1r_num4x4h[b.mi_size], n = bw4 * bh4, lb = ilog2p(bw4);
    for (int q = threadIdx.x & 15; q < n; q += 16) {
        const int r = b.mi_row + (q >> lb), c = b.mi_col + (q & (bw4 - 1));
        uint32_t* d = reinterpret_cast<uint32_t*>(const_cast<av1r_mi*>(k.mi) + (size_t)r * k.mi_stride + c);
#pragma unroll
        for (int i = 0; i < 6; i++) d[i] = w[i];
    }
}
// 16 lanes per transform block, one 4x4 unit each in turn (a 64x64 TB covers 256 units: one
// lane per TB serialised them behind its largest TB)
extern "C" __global__ __launch_bounds__(256) void k_mi_tbs(const KParams* kps)
{
    const KParams& k = KP(kps, blockIdx.y);
    const uint32_t ti = blockIdx.x * 16 + (threadIdx.x >> 4);
    if (ti >= k.n_tbs) return;
    const DevTb& t = k.tbs[ti];
    const int sub = t.plane ? 1 : 0;
    const int row = (t.y << sub) >> 2, col = (t.x << sub) >> 2;
    const int w4 = (av1r_tx_w[t.tx_size] >> 2) << sub, h4 = (av1r_tx_h[t.tx_size] >> 2) << sub;
    const int wIn = min(w4, k.mi_stride - col), hIn = min(h4, k.mi_rows_alloc - row);
    if (wIn <= 0 || hIn <= 0) return;
    uint8_t* base = reinterpret_cast<uint8_t*>(const_cast<av1r_mi*>(k.mi)) + offsetof(av1r_mi, lf_tx) + t.plane;
    const uint8_t v = t.tx_size;
    for (int q = threadIdx.x & 15; q < wIn * hIn; q += 16) {
        const int r = row + q / wIn, c = col + q % wIn;
        base[((size_t)r * k.mi_stride + c) * sizeof(av1r_mi)] = v;
    }
}
void launch_k_mi(const KParams* kps, int n, uint32_t maxUnits, uint32_t maxBlocks, uint32_t maxTbs, hipStream_t s)
{
    hipLaunchKernelGGL(k_mi_zero, dim3((maxUnits + 255) / 256, n), dim3(256), 0, s, kps);
    if (maxBlocks) hipLaunchKernelGGL(k_mi_blocks, dim3((maxBlocks + 15) / 16, n), dim3(256), 0, s, kps);
    if (maxTbs) hipLaunchKernelGGL(k_mi_tbs, dim3((maxTbs + 15) / 16, n), dim3(256), 0, s, kps);
}

// plain visible-region copy (stage snapshots)
extern "C" __global__ void k_copy_plane(DevPlane dst, DevPlane src)
{
    int x = blockIdx.x * 64 + (threadIdx.x & 63);
    int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x < src.w && y < src.h) dst.p[(size_t)y * dst.stride + x] = src.p[(size_t)y * src.stride + x];
}

// ------------------------------------------------------------------------------------
// k_stripe (round 6, A/B build -DAV1R_FUSED_STRIPE): deblocking -> CDEF
// -> loop restoration fused, one workgroup per (frame, LR stripe, run of 64-column tiles),
// walking its tiles left to right with every intermediate in LDS.  decode_frame_wrapup
// (Av1Decoder.cpp:181-189) runs the three filters over the whole frame in turn; what an LR
// stripe's output (rows [S, S + 64), S = 64 s - 8, LoopRestoration.cpp:136-189) depends on
// is bounded:
//   LR  rows [S, S + 64) reads CDEF rows [S, S + 64) and the deblocked rows S - 2, S - 1,
//       S + 64, S + 65 (get_source_sample, :234-246), 3 columns either side;
//   CDEF of the 8x8 blocks of rows [S, S + 64) (S is a multiple of 8) reads deblocked rows
//       [S - 2, S + 66), 2 columns either side (Cdef.cpp:158-198);
//   deblocking pass 1 (horizontal edges) writes at most 6 rows either side of an edge and reads
//       8: the edges y in [S - 4, S + 68] give rows [S - 2, S + 66), reading pass-0 rows
//       [S - 12, S + 76);
//   pass 0 (vertical edges) over those 88 rows; an edge writes 6 columns either side, reads 8.
// So the stripe's rows [S - 12, S + 76) are deblocked once (1.375x the stripe's rows, no
// horizontal recompute), with the stages lagging one another along the walk.  At the step for
// tile x0 (64 x0-aligned columns):
//   pass 0 for the vertical edges x in [x0, x0 + 64)      (reads [x0 - 8, x0 + 72))
//   pass 1 on columns [x0 - 8, x0 + 56)                   (pass 0 final left of x0 + 58)
//   CDEF of the 8x8 blocks of columns [x0 - 16, x0 + 48)  (reads deblocked [x0 - 18, x0 + 50))
//   LR of tile [x0 - 64, x0)                              (reads CDEF [x0 - 67, x0 + 3))
// in a window of columns [x0 - 80, x0 + 80) that moves by 64 after each step (chroma: half
// of everything; its LR stripe rows [S / 2, S / 2 + 32)).  A run of tiles [j0, j1) takes steps
// j0 - 1 .. j1 (the first and the last recompute one tile of deblocking and CDEF beside the
// run's neighbours).  The filters are the stage kernels' own device code: lf_edge / lf_unit
// on an LDS window, cdef_cost_f / cdef_quad, lr_filter_tile.  Reads the reconstructed frame
// (k.cur), writes the frame's output only (k.lrout, or k.cdef when the frame has no LR): no
// deblocked or CDEF frame in HBM.
// ------------------------------------------------------------------------------------
#ifdef AV1R_FUSED_STRIPE
#define FS_W 160          // luma window columns (x0 - 80 .. x0 + 80)
#define FS_CW 80          // chroma window columns
#define FS_DR 88          // deblocked luma rows (S - 12 .. S + 76)
#define FS_CDR 40         // deblocked chroma rows (S/2 - 4 .. S/2 + 36)
struct StripeLds {
    uint8_t dy[FS_DR][FS_W];          // luma: reconstruction -> deblocked, rows S - 12 ..
    uint8_t duv[2][FS_CDR][FS_CW];    // chroma, rows S/2 - 4 ..
    uint8_t cy[64][FS_W];             // CDEF output, luma rows S ..
    uint8_t cuv[2][32][FS_CW];        // chroma rows S/2 ..
    int cost[64][8];
    int16_t pri[64];
    uint8_t filt[64];
    int8_t idx[64];                   // the block's cdef_idx (-1: not filtered)
    int16_t offY[64][6], offC[64][6];
    LrLds lr;
};
DEV void fs_copy_row_dwords(uint8_t* dst, const uint8_t* src, int n4, int t0, int nt)
{
    for (int q = t0; q < n4; q += nt) reinterpret_cast<uint32_t*>(dst)[q] = reinterpret_cast<const uint32_t*>(src)[q];
}

extern "C" __global__ __launch_bounds__(256) void k_stripe(const KParams* kps, int nStripes, int runTiles, int nRuns)
{
    extern __shared__ __align__(16) uint8_t fs_smem[];
    StripeLds& L = *reinterpret_cast<StripeLds*>(fs_smem);
    const int t = threadIdx.x;
    const int per = nStripes * nRuns;
    const int f = blockIdx.x / per, rr = blockIdx.x - f * per;
    const int s = rr / nRuns, run = rr - s * nRuns;
    const KParams& k = KP(kps, f);
    const av1r_frame_hdr& h = *k.hdr;
    const int W = k.frame_w, H = k.frame_h;
    const int S = 64 * s - 8;
    if (S >= H) return;
    const int nTiles = (W + 63) / 64;
    const int j0 = run * runTiles, j1 = imin(nTiles, j0 + runTiles);
    if (j0 >= j1) return;
    const bool lfOn = h.lf_level[0] || h.lf_level[1];  // else LoopFilter::filter is skipped
    const int limX = k.mi_cols * 4, limY = k.mi_rows * 4, climX = k.mi_cols * 2, climY = k.mi_rows * 2;
    const DevPlane* R = k.cur.pl;
    const int Sc = S / 2;  // (S even: -8, 56, ...)
    for (int j = j0 - 1; j <= j1; j++) {
        const int x0 = 64 * j, cx0 = 32 * j;
        const int wx = x0 - 80, cwx = cx0 - 40;  // window origins
        // ---- the reconstruction of the new columns: [x0 + 8, x0 + 72) (the first step also
        // [x0 - 8, x0 + 8)), rows [S - 12, S + 76); outside the frame's allocation: 0
        {
            const int c0 = j == j0 - 1 ? 72 : 88, nc = (FS_W - 8 - c0) / 4;  // window columns c0 .. 152
            for (int q = t; q < FS_DR * nc; q += 256) {
                const int i = q / nc, d = q - i * nc, y = S - 12 + i, x = wx + c0 + 4 * d;
                uint32_t v = 0;
                if (y >= 0 && y < R[0].h + 64 && x >= 0 && x + 4 <= R[0].stride)
                    v = *reinterpret_cast<const uint32_t*>(R[0].p + (size_t)y * R[0].stride + x);
                *reinterpret_cast<uint32_t*>(&L.dy[i][c0 + 4 * d]) = v;
            }
            const int cc0 = c0 / 2, cnc = (FS_CW - 4 - cc0) / 4;  // chroma columns cc0 .. 76
            for (int q = t; q < 2 * FS_CDR * cnc; q += 256) {
                const int pl = q >= FS_CDR * cnc, r = q - pl * FS_CDR * cnc, i = r / cnc, d = r - i * cnc;
                const int y = Sc - 4 + i, x = cwx + cc0 + 4 * d;
                const DevPlane& P = R[1 + pl];
                uint32_t v = 0;
                if (y >= 0 && y < P.h + 32 && x >= 0 && x + 4 <= P.stride) v = *reinterpret_cast<const uint32_t*>(P.p + (size_t)y * P.stride + x);
                *reinterpret_cast<uint32_t*>(&L.duv[pl][i][cc0 + 4 * d]) = v;
            }
        }
        __syncthreads();
        const bool inFrame = x0 < W;
        // ---- deblocking pass 0: the vertical edges x in [x0, x0 + 64) of the window's rows
        if (lfOn && inFrame) {
            for (int q = t; q < 22 * 16 + 2 * 10 * 8; q += 256) {
                int plane, xP, yP, xT, yT;
                if (q < 22 * 16) {
                    const int ur = q >> 4, e = q & 15;
                    plane = 0, xP = x0 + 4 * e, yP = S - 12 + 4 * ur, xT = 80 + 4 * e, yT = 4 * ur;
                } else {
                    const int r2_ = q - 22 * 16, pl = r2_ / 80, r3 = r2_ - pl * 80, ur = r3 >> 3, e = r3 & 7;
                    plane = 1 + pl, xP = cx0 + 4 * e, yP = Sc - 4 + 4 * ur, xT = 40 + 4 * e, yT = 4 * ur;
                }
                LfEdge e;
                if (yP < 0 || !lf_edge(k, plane, 0, xP, yP, e)) continue;
                const LfLdsPx P{(lf_lds_u8*)(plane ? &L.duv[plane - 1][0][0] : &L.dy[0][0]), plane ? FS_CW : FS_W};
                lf_unit(P, plane, 0, xT, yT, e);
            }
        }
        __syncthreads();
        // ---- pass 1: the horizontal edges y in [S - 4, S + 68] on columns [x0 - 8, x0 + 56)
        // (chroma: edges [S/2, S/2 + 32] on [cx0 - 4, cx0 + 28))
        if (lfOn && x0 - 8 < W) {
            for (int q = t; q < 19 * 16 + 2 * 9 * 8; q += 256) {
                int plane, xP, yP, xT, yT;
                if (q < 19 * 16) {
                    const int er = q >> 4, u = q & 15;
                    plane = 0, xP = x0 - 8 + 4 * u, yP = S - 4 + 4 * er, xT = 72 + 4 * u, yT = 8 + 4 * er;
                } else {
                    const int r2_ = q - 19 * 16, pl = r2_ / 72, r3 = r2_ - pl * 72, er = r3 >> 3, u = r3 & 7;
                    plane = 1 + pl, xP = cx0 - 4 + 4 * u, yP = Sc + 4 * er, xT = 36 + 4 * u, yT = 4 + 4 * er;
                }
                LfEdge e;
                if (xP < 0 || yP < 0 || !lf_edge(k, plane, 1, xP, yP, e)) continue;
                const LfLdsPx P{(lf_lds_u8*)(plane ? &L.duv[plane - 1][0][0] : &L.dy[0][0]), plane ? FS_CW : FS_W};
                lf_unit(P, plane, 1, xT, yT, e);
            }
        }
        __syncthreads();
        // ---- CDEF of the 8x8 blocks of columns [x0 - 16, x0 + 48), rows [S, S + 64) (cdef_body
        // per block: its 64x64 region's cdef_idx, its skip test, direction, filter)
        const int bx0 = x0 - 16;
        if (bx0 < limX && j >= j0 - 1) {
            if (t < 64) {
                const int by = t >> 3, bxi = t & 7;
                const int yb = S + 8 * by, xb = bx0 + 8 * bxi;
                int idx = -1, fb = 0;
                if (yb >= 0 && yb < limY && xb >= 0 && xb < limX) {
                    const int mr = yb >> 2, mc = xb >> 2;
                    idx = k.cdef_idx[(mr >> 4) * h.cdef_cols + (mc >> 4)];
                    fb = !((mi_at(k, mr, mc).flags & AV1R_MI_SKIP) && (mi_at(k, mr + 1, mc).flags & AV1R_MI_SKIP) &&
                           (mi_at(k, mr, mc + 1).flags & AV1R_MI_SKIP) && (mi_at(k, mr + 1, mc + 1).flags & AV1R_MI_SKIP));
                }
                L.idx[t] = (int8_t)idx;
                L.filt[t] = (uint8_t)(idx != -1 && fb);
            }
            __syncthreads();
            {  // direction costs: wave w directions 2w, 2w + 1; lane = block
                const int b = t & 63, w = t >> 6;
                if (L.filt[b]) {
                    const int c = 64 + 8 * (b & 7), r = 12 + 8 * (b >> 3);  // window position (deblocked rows from S - 12)
                    uint32_t rw[8][2];
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        const uint2 v = *reinterpret_cast<const uint2*>(&L.dy[r + i][c]);
                        rw[i][0] = v.x;
                        rw[i][1] = v.y;
                    }
                    auto px8 = [&](int i, int jj) { return (int)((rw[i][jj >> 2] >> (8 * (jj & 3))) & 0xff) - 128; };
                    int c0_, c1_;
                    switch (__builtin_amdgcn_readfirstlane(w)) {
                    case 0: c0_ = cdef_cost_f<0>(px8), c1_ = cdef_cost_f<1>(px8); break;
                    case 1: c0_ = cdef_cost_f<2>(px8), c1_ = cdef_cost_f<3>(px8); break;
                    case 2: c0_ = cdef_cost_f<4>(px8), c1_ = cdef_cost_f<5>(px8); break;
                    default: c0_ = cdef_cost_f<6>(px8), c1_ = cdef_cost_f<7>(px8); break;
                    }
                    L.cost[b][2 * w] = c0_;
                    L.cost[b][2 * w + 1] = c1_;
                }
            }
            __syncthreads();
            if (t < 64 && L.filt[t]) {
                const int idx = L.idx[t];
                int best = 0, yDir = 0;
                for (int d = 0; d < 8; d++)
                    if (L.cost[t][d] > best) {
                        best = L.cost[t][d];
                        yDir = d;
                    }
                const int var = (best - L.cost[t][(yDir + 4) & 7]) >> 10;
                const int priStr = h.cdef_y_pri[idx];
                const int varStr = (var >> 6) ? imin(floor_log2(var >> 6), 12) : 0;
                L.pri[t] = (int16_t)(var ? (priStr * (4 + varStr) + 8) >> 4 : 0);
                const int dy0 = priStr == 0 ? 0 : yDir, dc0 = h.cdef_uv_pri[idx] == 0 ? 0 : av1r_cdef_uv_dir420[yDir];
#pragma unroll
                for (int ss = 0; ss < 3; ss++)
#pragma unroll
                    for (int kk = 0; kk < 2; kk++) {
                        const int dl = ss == 0 ? dy0 : ((dy0 + (ss == 1 ? -2 : 2)) & 7);
                        const int dc = ss == 0 ? dc0 : ((dc0 + (ss == 1 ? -2 : 2)) & 7);
                        L.offY[t][ss * 2 + kk] = (int16_t)(av1r_cdef_directions[dl][kk][0] * FS_W + av1r_cdef_directions[dl][kk][1]);
                        L.offC[t][ss * 2 + kk] = (int16_t)(av1r_cdef_directions[dc][kk][0] * FS_CW + av1r_cdef_directions[dc][kk][1]);
                    }
            }
            __syncthreads();
            // luma: 64 rows x 16 four-pixel groups = 1024 groups, 4 per lane; a group's block is
            // (row >> 3, group >> 1)
            for (int q = t; q < 1024; q += 256) {
                const int i = q >> 4, g = q & 15, b = (i >> 3) * 8 + (g >> 1);
                const int y = S + i, x = bx0 + 4 * g;
                if (y < 0 || y >= limY || x >= limX || x < 0) continue;
                const int p = (12 + i) * FS_W + 64 + 4 * g;
                uint32_t o;
                if (!L.filt[b]) o = *reinterpret_cast<const uint32_t*>(&L.dy[0][0] + p);
                else o = cdef_quad<true>(&L.dy[0][0], p, L.offY[b], L.pri[b], h.cdef_y_sec[L.idx[b]], h.cdef_damping, x, y, FS_W, limX, limY);
                *reinterpret_cast<uint32_t*>(&L.cy[i][64 + 4 * g]) = o;
            }
            // chroma: 2 planes x 32 rows x 8 groups (a 4x4 block per group column, its luma block's
            // direction and strengths)
            for (int q = t; q < 512; q += 256) {
                const int pl = q >> 8, r = q & 255, i = r >> 3, g = r & 7, b = (i >> 2) * 8 + g;
                const int y = Sc + i, x = bx0 / 2 + 4 * g;
                if (y < 0 || y >= climY || x >= climX || x < 0) continue;
                const uint8_t* tile = &L.duv[pl][0][0];
                const int p = (4 + i) * FS_CW + 32 + 4 * g;
                uint32_t o;
                if (!L.filt[b]) {
                    o = *reinterpret_cast<const uint32_t*>(tile + p);
                } else {
                    const int idx = L.idx[b];
                    o = cdef_quad<true>(tile, p, L.offC[b], h.cdef_uv_pri[idx], h.cdef_uv_sec[idx], h.cdef_damping - 1, x, y, FS_CW,
                        climX, climY);
                }
                *reinterpret_cast<uint32_t*>(&L.cuv[pl][i][32 + 4 * g]) = o;
            }
        }
        __syncthreads();
        // ---- LR (or the CDEF output as it is) of tile j - 1: columns [x0 - 64, x0)
        if (j - 1 >= j0) {
            const int lx0 = x0 - 64;
#pragma unroll 1
            for (int part = 0; part < 4; part++) {  // luma rows [S, S + 32), [S + 32, S + 64); U; V
                const int plane = part < 2 ? 0 : part - 1, sub = plane ? 1 : 0;
                const DevPlane O = h.uses_lr ? k.lrout.pl[plane] : k.cdef.pl[plane];
                const int pw = O.w, ph = O.h;
                const int tx0 = lx0 >> sub, tw = imin(64 >> sub, pw - tx0);
                const int start = plane ? Sc : S, end = start + (64 >> sub);
                const int ty0 = imax(0, plane ? start : start + 32 * part), ty1 = imin(plane ? end : start + 32 * (part + 1), ph);
                if (tw <= 0 || ty0 >= ty1) continue;
                const int th = ty1 - ty0;
                const uint8_t* cw_ = plane ? &L.cuv[plane - 1][0][0] : &L.cy[0][0];
                const uint8_t* dw_ = plane ? &L.duv[plane - 1][0][0] : &L.dy[0][0];
                const int ws = plane ? FS_CW : FS_W, wox = plane ? cwx : wx;
                const int dRow0 = plane ? Sc - 4 : S - 12;  // the deblocked window's first row
                if (!h.uses_lr || h.lr_type[plane] == AV1R_RESTORE_NONE) {
                    for (int q = t; q < th * tw; q += 256) {
                        const int r = q / tw, c = q - r * tw;
                        O.p[(size_t)(ty0 + r) * O.stride + tx0 + c] = cw_[(ty0 + r - start) * ws + tx0 + c - wox];
                    }
                    continue;
                }
                // stage L.src: rows ty0 - 3 .. ty1 + 2, columns tx0 - 4 .. tx0 + 67 (get_source_sample:
                // CDEF rows inside the stripe, deblocked rows S - 2, S - 1 / end, end + 1 outside;
                // coordinates clamped to the plane)
                for (int q = t; q < (th + 6) * LR_SW; q += 256) {
                    const int i = q / LR_SW, jj = q - i * LR_SW;
                    int y = ty0 - 3 + i;
                    const bool pre = y < start || y >= end;
                    if (y < start) y = imax(start - 2, y);
                    else if (y >= end) y = imin(end + 1, y);
                    y = CLIP3(0, ph - 1, y);
                    const int x = CLIP3(0, pw - 1, tx0 - 4 + jj) - wox;
                    L.lr.src[i][jj] = pre ? dw_[(y - dRow0) * ws + x] : cw_[(y - start) * ws + x];
                }
                const int us = h.lr_unit_size[plane], rows = h.lr_unit_rows[plane], cols = h.lr_unit_cols[plane];
                const int off = 8 >> sub;
                const int ur = imin((ty0 + off) / us, rows - 1);
                const int uc0 = imin(tx0 / us, cols - 1);
                const int nU = imin((tx0 + tw - 1) / us, cols - 1) - uc0 + 1;
                if (t < nU) L.lr.unit[t] = k.lr[h.lr_unit_off[plane] + ur * cols + uc0 + t];
                __syncthreads();
                lr_filter_tile(L.lr, h, plane, tx0, tw, ty0, th, imax(start, 0), us, cols, uc0, nU, r2(k.frame_w, sub),
                    r2(k.frame_h, sub), O);
                __syncthreads();
            }
        }
        // ---- the windows move by one tile: columns [64, 160) -> [0, 96) (chroma [32, 80) -> [0, 48))
        {
            constexpr int NL = FS_DR * 24 + 64 * 24, NC = 2 * (FS_CDR * 12 + 32 * 12);  // dwords
            uint32_t v[(NL + NC + 255) / 256];
#pragma unroll
            for (int u = 0; u < (NL + NC + 255) / 256; u++) {
                const int q = t + 256 * u;
                uint32_t* src = nullptr;
                if (q < FS_DR * 24) src = reinterpret_cast<uint32_t*>(&L.dy[q / 24][64 + 4 * (q % 24)]);
                else if (q < NL) { const int r = q - FS_DR * 24; src = reinterpret_cast<uint32_t*>(&L.cy[r / 24][64 + 4 * (r % 24)]); }
                else if (q < NL + NC) {
                    int r = q - NL;
                    const int pl = r / (FS_CDR * 12 + 32 * 12);
                    r -= pl * (FS_CDR * 12 + 32 * 12);
                    src = r < FS_CDR * 12 ? reinterpret_cast<uint32_t*>(&L.duv[pl][r / 12][32 + 4 * (r % 12)])
                                          : reinterpret_cast<uint32_t*>(&L.cuv[pl][(r - FS_CDR * 12) / 12][32 + 4 * ((r - FS_CDR * 12) % 12)]);
                }
                v[u] = src ? *src : 0u;
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < (NL + NC + 255) / 256; u++) {
                const int q = t + 256 * u;
                uint32_t* dst = nullptr;
                if (q < FS_DR * 24) dst = reinterpret_cast<uint32_t*>(&L.dy[q / 24][4 * (q % 24)]);
                else if (q < NL) { const int r = q - FS_DR * 24; dst = reinterpret_cast<uint32_t*>(&L.cy[r / 24][4 * (r % 24)]); }
                else if (q < NL + NC) {
                    int r = q - NL;
                    const int pl = r / (FS_CDR * 12 + 32 * 12);
                    r -= pl * (FS_CDR * 12 + 32 * 12);
                    dst = r < FS_CDR * 12 ? reinterpret_cast<uint32_t*>(&L.duv[pl][r / 12][4 * (r % 12)])
                                          : reinterpret_cast<uint32_t*>(&L.cuv[pl][(r - FS_CDR * 12) / 12][4 * ((r - FS_CDR * 12) % 12)]);
                }
                if (dst) *dst = v[u];
            }
            __syncthreads();
        }
    }
}
void launch_k_stripe(const KParams* kps, int n, int maxW, int maxH, int runTiles, hipStream_t s)
{
    const int nStripes = (maxH + 8 + 63) / 64, nTiles = (maxW + 63) / 64;
    const int nRuns = (nTiles + runTiles - 1) / runTiles;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_stripe), hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(StripeLds));
        attr = true;
    }
    hipLaunchKernelGGL(k_stripe, dim3(n * nStripes * nRuns), dim3(256), sizeof(StripeLds), s, kps, nStripes, runTiles, nRuns);
}
#endif  // AV1R_FUSED_STRIPE

// ------------------------------------------------------------------------------------
// launches over n frames: grid row / slice per frame, sized for the largest
void launch_k_lf(const KParams* kps, int n, int pass, int maxUnits, hipStream_t s)
{
    hipLaunchKernelGGL(k_lf, dim3((maxUnits + 255) / 256, n), dim3(256), 0, s, kps, pass);
}
void launch_k_cdef(const KParams* kps, int n, int maxMiCols, int maxMiRows, hipStream_t s)
{
    hipLaunchKernelGGL(k_cdef, dim3((maxMiCols + 15) / 16, (maxMiRows + 15) / 16, n), dim3(256), 0, s, kps);
}
void launch_k_lr(const KParams* kps, int n, int maxW, int maxH, hipStream_t s)
{
    // tile rows: luma stripes (64 rows from -8) in halves; chroma stripes whole
    const int tilesY = 2 * ((maxH + 8 + 63) / 64);
    const int nxl = (maxW + LR_TW - 1) / LR_TW, nxc = ((maxW + 1) / 2 + LR_TW - 1) / LR_TW;
    const int nyc = ((maxH + 1) / 2 + 4 + 31) / 32;  // chroma stripes (32 rows from -4)
    hipLaunchKernelGGL(k_lr, dim3(n * (nxl * tilesY + 2 * nxc * nyc)), dim3(256), 0, s, kps, nxl, tilesY, nxc, nyc);
}
void launch_k_copy_plane(const DevPlane& dst, const DevPlane& src, hipStream_t s)
{
    hipLaunchKernelGGL(k_copy_plane, dim3((src.w + 63) / 64, (src.h + 3) / 4), dim3(256), 0, s, dst, src);
}
