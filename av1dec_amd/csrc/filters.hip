// filters.hip -- in-loop post-filters for gfx950: deblocking, CDEF, loop restoration.
//
//   k_lf    one lane per 4x4 edge unit (all planes, one pass per launch): LoopFilter::
//           loop_filter_edge + sampleFilter/narrowFilter/wideFilter
//           (decoder/LoopFilter.cpp:85-289).  Edges of one pass never overlap their
//           read/write footprints (the filter length is bounded by the transform sizes
//           on both sides), so a pass is embarrassingly parallel, in place.
//   k_cdef  one wave per 8x8 luma block, lane = pixel: Cdef::cdef_block (Cdef.cpp:72-101),
//           cdefDirection via LDS partial sums (:203-261), cdefFilter (:158-198) into a
//           separate output frame (blocks that are skipped are copied).
//   k_lr    one lane per output pixel: LoopRestoration Wiener (LoopRestoration.cpp:247-277)
//           and self-guided (:284-479) with the stripe/unit geometry of :33-189; the
//           3-pixel border extension (:196-198) is coordinate clamping.
#include "av1r_dev.h"

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

DEV void lf_sample(const DevPlane& P, int x, int y, int plane, int limit, int blimit, int thresh, int dx, int dy, int filterSize)
{
    uint8_t* c = P.p + (size_t)y * P.stride + x;
    const int step = dx + dy * P.stride;
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
    const int log2Size = (filterSize == 8 || !flat2) ? 3 : 4;
    const int n = log2Size == 4 ? 6 : (!plane ? 3 : 2);
    const int n2 = (log2Size == 3 && !plane) ? 0 : 1;
    int v[14];  // v[p + 7] = pixel at offset p, p in [-7, 6]
#pragma unroll
    for (int p = -7; p <= 6; p++) v[p + 7] = (p >= -(n + 1) && p <= n) ? c[step * p] : 0;
    int F[12];
    for (int i = -n; i < n; i++) {
        int t = 0;
        for (int j = -n; j <= n; j++) {
            int p = CLIP3(-(n + 1), n, i + j);
            t += v[p + 7] * ((iabs(j) <= n2) ? 2 : 1);
        }
        F[i + n] = r2(t, log2Size);
    }
    for (int i = -n; i < n; i++) c[step * i] = (uint8_t)F[i + n];
#undef PP
#undef QQ
}

// one lane per (plane, 4x4 unit) edge of pass `pass`
extern "C" __global__ __launch_bounds__(256) void k_lf(KParams k, int pass, int nY, int nC, int cCols, int planeMask)
{
    int id = blockIdx.x * blockDim.x + threadIdx.x;
    int plane, row0, col0;
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
        return;
    }
    if (!((planeMask >> plane) & 1)) return;
    const int sub = plane ? 1 : 0;
    const int dx = pass == 0, dy = pass == 1;
    const int x = col0 * 4, y = row0 * 4;
    const int row = row0 | sub, col = col0 | sub;
    if (x >= k.frame_w || y >= k.frame_h) return;
    if (!pass && !x) return;
    if (pass && !y) return;
    const int xP = x >> sub, yP = y >> sub;
    const int prevRow = row - (dy << sub), prevCol = col - (dx << sub);
    const av1r_mi& info = mi_at(k, row, col);
    const int txSz = info.lf_tx[plane];
    const int psz = plane_bsize(info.mi_size, plane);
    const int skip = info.flags & AV1R_MI_SKIP;
    const int isIntra = info.ref_frame[0] <= AV1R_INTRA_FRAME;
    const int prevTx = mi_at(k, prevRow, prevCol).lf_tx[plane];
    const int isBlockEdge = !pass ? !(xP % (av1r_num4x4w[psz] * 4)) : !(yP % (av1r_num4x4h[psz] * 4));
    const int isTxEdge = !pass ? !(xP % av1r_tx_w[txSz]) : !(yP % av1r_tx_h[txSz]);
    if (!(isTxEdge && (isBlockEdge || !skip || isIntra))) return;
    const int base = !pass ? imin(av1r_tx_w[prevTx], av1r_tx_w[txSz]) : imin(av1r_tx_h[prevTx], av1r_tx_h[txSz]);
    const int filterSize = !plane ? imin(16, base) : imin(8, base);
    int lvl = lf_level(k, row, col, plane, pass);
    if (!lvl) lvl = lf_level(k, prevRow, prevCol, plane, pass);
    if (lvl <= 0) return;
    const int sharp = k.hdr->lf_sharpness;
    const int shift = sharp > 4 ? 2 : (sharp > 0 ? 1 : 0);
    const int limit = sharp > 0 ? CLIP3(1, 9 - sharp, lvl >> shift) : imax(1, lvl >> shift);
    const int blimit = 2 * (lvl + 2) + limit;
    const int thresh = lvl >> 4;
    const DevPlane& P = k.cur.pl[plane];
    for (int i = 0; i < 4; i++) lf_sample(P, xP + dy * i, yP + dx * i, plane, limit, blimit, thresh, dx, dy, filterSize);
}

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

DEV void cdef_plane(const KParams& k, int plane, int r, int c, int priStr, int secStr, int damping, int dir, int i, int j)
{
    const int sub = plane ? 1 : 0;
    const DevPlane& in = k.cur.pl[plane];
    const int x0 = (c * 4) >> sub, y0 = (r * 4) >> sub;
    const int X = x0 + j, Y = y0 + i;
    const int x = px(in, X, Y);
    int sum = 0, mx = x, mn = x;
#pragma unroll
    for (int kk = 0; kk < 2; kk++)
#pragma unroll
        for (int sgn = -1; sgn <= 1; sgn += 2)
#pragma unroll
            for (int s = 0; s < 3; s++) {
                int d = s == 0 ? dir : ((dir + (s == 1 ? -2 : 2)) & 7);
                int yy = Y + sgn * av1r_cdef_directions[d][kk][0];
                int xx = X + sgn * av1r_cdef_directions[d][kk][1];
                int cr = (yy << sub) >> 2, cc = (xx << sub) >> 2;
                if (!(cc >= 0 && cc < k.mi_cols && cr >= 0 && cr < k.mi_rows)) continue;
                int p = px(in, xx, yy);
                if (s == 0) sum += av1r_cdef_pri_taps[priStr & 1][kk] * constrain(p - x, priStr, damping);
                else sum += av1r_cdef_sec_taps[priStr & 1][kk] * constrain(p - x, secStr, damping);
                mx = imax(p, mx);
                mn = imin(p, mn);
            }
    px(k.out.pl[plane], X, Y) = (uint8_t)CLIP3(mn, mx, x + ((8 + sum - (sum < 0)) >> 4));
}

// one wave per 8x8 luma block (lane = luma pixel; lanes 0..31 also do the 4x4 U/V)
extern "C" __global__ __launch_bounds__(256) void k_cdef(KParams k, int nBlocks, int bCols)
{
    __shared__ int partial[4][8][16];
    __shared__ int cost[4][8];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + wv;
    const bool active = b < nBlocks;
    const int r = active ? (b / bCols) * 2 : 0, c = active ? (b % bCols) * 2 : 0;
    const int i = lane >> 3, j = lane & 7;
    int idx = -1, skip = 1;
    if (active) {
        idx = k.cdef_idx[(r >> 4) * k.hdr->cdef_cols + (c >> 4)];
        skip = (mi_at(k, r, c).flags & AV1R_MI_SKIP) && (mi_at(k, r + 1, c).flags & AV1R_MI_SKIP)
            && (mi_at(k, r, c + 1).flags & AV1R_MI_SKIP) && (mi_at(k, r + 1, c + 1).flags & AV1R_MI_SKIP);
    }
    const bool filt = active && idx != -1 && !skip;
    // the reference filters into a copy of the frame (Cdef.cpp:43): unfiltered blocks copy
    if (active && !filt) {
        px(k.out.pl[0], c * 4 + j, r * 4 + i) = px(k.cur.pl[0], c * 4 + j, r * 4 + i);
        if (lane < 32) {
            int pl = 1 + (lane >> 4), q = lane & 15;
            px(k.out.pl[pl], c * 2 + (q & 3), r * 2 + (q >> 2)) = px(k.cur.pl[pl], c * 2 + (q & 3), r * 2 + (q >> 2));
        }
    }
    for (int q = lane; q < 8 * 16; q += 64) partial[wv][q >> 4][q & 15] = 0;
    __syncthreads();
    int x = 0;
    if (filt) {
        x = px(k.cur.pl[0], c * 4 + j, r * 4 + i) - 128;
        atomicAdd(&partial[wv][0][i + j], x);
        atomicAdd(&partial[wv][1][i + j / 2], x);
        atomicAdd(&partial[wv][2][i], x);
        atomicAdd(&partial[wv][3][3 + i - j / 2], x);
        atomicAdd(&partial[wv][4][7 + i - j], x);
        atomicAdd(&partial[wv][5][3 - i / 2 + j], x);
        atomicAdd(&partial[wv][6][j], x);
        atomicAdd(&partial[wv][7][i / 2 + j], x);
    }
    __syncthreads();
    if (filt && lane < 8) {
        // cdefDirection costs (Cdef.cpp:229-253), lane = direction
        const int d = lane;
        const int* pp = partial[wv][d];
        int cst = 0;
        if (d == 2 || d == 6) {
            for (int q = 0; q < 8; q++) cst += pp[q] * pp[q];
            cst *= av1r_cdef_div_table[8];
        } else if (d == 0 || d == 4) {
            for (int q = 0; q < 7; q++) cst += (pp[q] * pp[q] + pp[14 - q] * pp[14 - q]) * av1r_cdef_div_table[q + 1];
            cst += pp[7] * pp[7] * av1r_cdef_div_table[8];
        } else {
            for (int q = 0; q < 5; q++) cst += pp[3 + q] * pp[3 + q];
            cst *= av1r_cdef_div_table[8];
            for (int q = 0; q < 3; q++) cst += (pp[q] * pp[q] + pp[10 - q] * pp[10 - q]) * av1r_cdef_div_table[2 * q + 2];
        }
        cost[wv][d] = cst;
    }
    __syncthreads();
    if (!filt) return;
    int best = 0, yDir = 0;
    for (int d = 0; d < 8; d++)
        if (cost[wv][d] > best) {
            best = cost[wv][d];
            yDir = d;
        }
    const int var = (best - cost[wv][(yDir + 4) & 7]) >> 10;
    const av1r_frame_hdr& h = *k.hdr;
    int priStr = h.cdef_y_pri[idx], secStr = h.cdef_y_sec[idx];
    int dir = priStr == 0 ? 0 : yDir;
    int varStr = (var >> 6) ? imin(floor_log2(var >> 6), 12) : 0;
    priStr = var ? (priStr * (4 + varStr) + 8) >> 4 : 0;
    cdef_plane(k, 0, r, c, priStr, secStr, h.cdef_damping, dir, i, j);
    if (lane < 32) {
        int pl = 1 + (lane >> 4), q = lane & 15;
        int uvPri = h.cdef_uv_pri[idx], uvSec = h.cdef_uv_sec[idx];
        int uvDir = uvPri == 0 ? 0 : av1r_cdef_uv_dir420[yDir];
        cdef_plane(k, pl, r, c, uvPri, uvSec, h.cdef_damping - 1, uvDir, q >> 2, q & 3);
    }
}

// ------------------------------------------------------------------------------------
// Loop restoration
// ------------------------------------------------------------------------------------
struct LrPix {
    DevPlane cdefP;  // CDEF output (k.cur)
    DevPlane preP;   // deblocked, pre-CDEF frame (k.ref[0] slot reused by the host)
    int start, end;  // stripe
};
// get_source_sample (LoopRestoration.cpp:234-246) + extendBorder(3) as clamping
DEV int lr_src(const LrPix& S, int x, int y)
{
    const bool pre = y < S.start || y >= S.end;
    if (y < S.start) y = imax(S.start - 2, y);
    else if (y >= S.end) y = imin(S.end + 1, y);
    const DevPlane& P = pre ? S.preP : S.cdefP;
    x = CLIP3(0, P.w - 1, x);
    y = CLIP3(0, P.h - 1, y);
    return P.p[(size_t)y * P.stride + x];
}

DEV void sgr_ab(const LrPix& S, int x, int y, int r, int set, int pass, int& A, int& B)
{
    int eps = av1r_sgr_params[set][pass * 2 + 1];
    int n = (2 * r + 1) * (2 * r + 1);
    int n2e = n * n * eps;
    int s = ((1 << 20) + n2e / 2) / n2e;
    int a = 0, b = 0;
    for (int dy = -r; dy <= r; dy++)
        for (int dx = -r; dx <= r; dx++) {
            int cv = lr_src(S, x + dx, y + dy);
            a += cv * cv;
            b += cv;
        }
    int p = imax(0, a * n - b * b);
    int z = (int)((uint32_t)p * (uint32_t)s + (1u << 19)) >> 20;
    int a2;
    if (z >= 255) a2 = 256;
    else if (z == 0) a2 = 1;
    else a2 = ((z << 8) + (z / 2)) / (z + 1);
    int oneOverN = ((1 << 12) + (n / 2)) / n;
    int b2 = ((1 << 8) - a2) * b * oneOverN;
    A = a2;
    B = r2(b2, 12);
}

// boxFilter output for pixel (x, y) = row i of the block that starts at row y0
DEV int sgr_filter(const LrPix& S, const DevPlane& cdefP, int x, int y, int i, int set, int pass, int r)
{
    int shift = (pass == 0 && (i & 1)) ? 4 : 5;
    int a = 0, b = 0;
    for (int dy = -1; dy <= 1; dy++) {
        if (pass == 0 && !((i + dy) & 1)) continue;
        for (int dx = -1; dx <= 1; dx++) {
            int wt = pass == 0 ? (dx == 0 ? 6 : 5) : ((dx == 0 || dy == 0) ? 4 : 3);
            int A, B;
            sgr_ab(S, x + dx, y + dy, r, set, pass, A, B);
            a += wt * A;
            b += wt * B;
        }
    }
    int v = a * cdefP.p[(size_t)y * cdefP.stride + x] + b;
    return r2(v, 8 + shift - 4);
}

// one lane per visible pixel, all planes in one launch (blockIdx.z = plane);
// k.cur = CDEF frame, k.ref[0] = deblocked frame, k.out = restored frame.
extern "C" __global__ __launch_bounds__(256) void k_lr(KParams k)
{
    const int plane = blockIdx.z;
    const DevPlane C = k.cur.pl[plane];
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= C.w || y >= C.h) return;
    const av1r_frame_hdr& h = *k.hdr;
    const int sub = plane ? 1 : 0;
    uint8_t outv = C.p[(size_t)y * C.stride + x];
    if (h.lr_type[plane] != AV1R_RESTORE_NONE) {
        const int us = h.lr_unit_size[plane];
        const int rows = h.lr_unit_rows[plane], cols = h.lr_unit_cols[plane];
        const int off = 8 >> sub;
        const int planeEndX = r2(k.frame_w, sub), planeEndY = r2(k.frame_h, sub);
        if (x < planeEndX && y < planeEndY) {
            int uc = imin(x / us, cols - 1);
            int ur = imin((y + off) / us, rows - 1);
            const av1r_lr_unit& u = k.lr[h.lr_unit_off[plane] + ur * cols + uc];
            if (u.type != AV1R_RESTORE_NONE) {
                int uy = ur * us;
                if (uy) uy -= off;
                int stripeNum = (y + off) / (64 >> sub);
                LrPix S;
                S.cdefP = C;
                S.preP = k.ref[0].pl[plane];
                S.start = (-8 + stripeNum * 64) >> sub;
                S.end = S.start + (64 >> sub);
                const int y0 = imax(S.start, uy);  // forEachBlock's y
                if (u.type == AV1R_RESTORE_WIENER) {
                    int vf[7], hf[7];
                    vf[3] = hf[3] = 128;
                    for (int q = 0; q < 3; q++) {
                        vf[q] = vf[6 - q] = u.wiener[0][q];
                        hf[q] = hf[6 - q] = u.wiener[1][q];
                        vf[3] -= 2 * u.wiener[0][q];
                        hf[3] -= 2 * u.wiener[1][q];
                    }
                    const int offset = 1 << (8 + 7 - 3 - 1), limit = (1 << (8 + 1 + 7 - 3)) - 1;
                    int s = 0;
                    for (int t = 0; t < 7; t++) {
                        int hs = 0;
                        for (int q = 0; q < 7; q++) hs += hf[q] * lr_src(S, x + q - 3, y + t - 3);
                        int v = CLIP3(-offset, limit - offset, r2(hs, 3));
                        s += vf[t] * v;
                    }
                    outv = (uint8_t)clip1(r2(s, 11));
                } else {
                    const int set = u.sgr_set;
                    const int r0 = av1r_sgr_params[set][0], r1 = av1r_sgr_params[set][2];
                    const int i = y - y0;
                    int uu = C.p[(size_t)y * C.stride + x] << 4;
                    int w0 = u.sgr_xqd[0], w1 = u.sgr_xqd[1], w2 = (1 << 7) - w0 - w1;
                    int v = w1 * uu;
                    v += r0 ? w0 * sgr_filter(S, C, x, y, i, set, 0, r0) : w0 * uu;
                    v += r1 ? w2 * sgr_filter(S, C, x, y, i, set, 1, r1) : w2 * uu;
                    outv = (uint8_t)clip1(r2(v, 4 + 7));
                }
            }
        }
    }
    k.out.pl[plane].p[(size_t)y * k.out.pl[plane].stride + x] = outv;
}

// plain visible-region copy (stage snapshots)
extern "C" __global__ void k_copy_plane(DevPlane dst, DevPlane src)
{
    int x = blockIdx.x * 64 + (threadIdx.x & 63);
    int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x < src.w && y < src.h) dst.p[(size_t)y * dst.stride + x] = src.p[(size_t)y * src.stride + x];
}

// ------------------------------------------------------------------------------------
void launch_k_lf(const KParams& k, int pass, int nY, int nC, int cCols, int planeMask, hipStream_t s)
{
    int n = nY + 2 * nC;
    hipLaunchKernelGGL(k_lf, dim3((n + 255) / 256), dim3(256), 0, s, k, pass, nY, nC, cCols, planeMask);
}
void launch_k_cdef(const KParams& k, int nBlocks, int bCols, hipStream_t s)
{
    hipLaunchKernelGGL(k_cdef, dim3((nBlocks + 3) / 4), dim3(256), 0, s, k, nBlocks, bCols);
}
void launch_k_lr(const KParams& k, hipStream_t s)
{
    const DevPlane& p = k.cur.pl[0];
    hipLaunchKernelGGL(k_lr, dim3((p.w + 63) / 64, (p.h + 3) / 4, 3), dim3(256), 0, s, k);
}
void launch_k_copy_plane(const DevPlane& dst, const DevPlane& src, hipStream_t s)
{
    hipLaunchKernelGGL(k_copy_plane, dim3((src.w + 63) / 64, (src.h + 3) / 4), dim3(256), 0, s, dst, src);
}
