// intra_fast.h -- the dataflow kernels' lean path for small intra transform blocks.
//
// k_flow items are chains: a transform block's prediction waits for its
// neighbours' pixels, and a key frame is ~2 000 such hops deep, so what counts is the
// time from "edges arrived" to "pixels published".  The generic path (tb_predict +
// coop_intra_from_edges + tb_store_flow, written for any NT and any size) spent ~1 200
// instructions per 4x4 block there, most of them scalar control flow deriving the
// prediction parameters.  This path, for one wave and w, h <= 16 (k_flow's small items):
//   fi_setup  -- BEFORE the dependency wait: every parameter (mode class, angle, edge
//                filter strengths and lengths, upsampling, dx / dy, limits), all uniform;
//   fi_run    -- after it: the edge units (gran_gather) -> one pass building AboveRow /
//                LeftCol (edge filter and corner filter folded in) -> one upsampling
//                pass -> four pixels per lane -> add the residual -> store, granules
//                straight from the registers.
// Restates IntraPredict::predict_intra (decoder/IntraPredict.cpp:563-630) with the
// directional predictor (:379-483, edge preparation :394-437, filterCorner :204-209,
// intraEdgeFilter :324-337, upsampling :354-370), dcPredict (:485-508), smoothPredict
// (:510-561), paethPredict (:151-171) and predict_chroma_from_luma (:632-667), as
// intra_dev.h does; palette and filter-intra blocks keep the generic path.
#pragma once
#include "intra_dev.h"

// (the prediction classes FI_* are in av1r_dev.h: the host writes them into TinyItem)

struct FiParams {
    int cls;
    int log2W, log2H;
    bool hA, hL, cfl;
    int aboveLimit, leftLimit;  // as coop_intra_edges
    int strA, strL, nA, nL;     // edge filter strengths (0: none) and lengths (numPx + 1)
    int nUA, nUL;               // upsampled lengths (0: no upsampling)
    int corner;                 // filterCorner
    int dx, dy;
    int alpha;                  // CFL
    int maxLW, maxLH;
};

// the lean path takes this item: an intra TB (not palette) of a one-wave item, no filter-intra
DEV bool fi_ok(const WorkItem& tb, const DevBlock& blk)
{
    return tb.pred == AV1R_PRED_INTRA && !(tb.plane == 0 && (blk.flags & AV1R_BLK_FILTER_INTRA));
}

// Every parameter of the prediction (uniform: scalar registers), from the batch only
DEV FiParams fi_setup(const KParams& k, const WorkItem& tb, const DevBlock& blk, int edgeFilter)
{
    FiParams F;
    const int plane = tb.plane, x = tb.x, y = tb.y, sub = plane ? 1 : 0;
    F.log2W = stab(av1r_tx_w_log2, tb.tx_size);
    F.log2H = stab(av1r_tx_h_log2, tb.tx_size);
    const int w = 1 << F.log2W, h = 1 << F.log2H;
    const int maxXd = (k.mi_cols * 4) >> sub, maxYd = (k.mi_rows * 4) >> sub;
    F.hA = (tb.flags & AV1R_TB_HAVE_ABOVE) != 0;
    F.hL = (tb.flags & AV1R_TB_HAVE_LEFT) != 0;
    F.aboveLimit = imin(maxXd - 1, x + ((tb.flags & AV1R_TB_HAVE_AR) ? 2 * w : w) - 1);
    F.leftLimit = imin(maxYd - 1, y + ((tb.flags & AV1R_TB_HAVE_BL) ? 2 * h : h) - 1);
    F.cfl = plane > 0 && blk.uv_mode == AV1R_UV_CFL_PRED;
    F.alpha = plane == 1 ? blk.cfl_alpha_u : blk.cfl_alpha_v;
    F.maxLW = blk.max_luma_w;
    F.maxLH = blk.max_luma_h;
    const int mode = plane == 0 ? blk.y_mode : (F.cfl ? AV1R_DC_PRED : blk.uv_mode);
    const int smooth = plane ? ((blk.flags & (AV1R_BLK_SMOOTH_A_UV | AV1R_BLK_SMOOTH_L_UV)) != 0)
                             : ((blk.flags & (AV1R_BLK_SMOOTH_A_Y | AV1R_BLK_SMOOTH_L_Y)) != 0);
    F.strA = F.strL = F.nA = F.nL = F.nUA = F.nUL = F.corner = F.dx = F.dy = 0;
    if (mode >= AV1R_V_PRED && mode <= AV1R_D67_PRED) {
        const int pAngle = stab(av1r_mode_to_angle, mode) + (plane == 0 ? blk.angle_delta_y : blk.angle_delta_uv) * 3;
        F.cls = pAngle < 90 ? FI_Z1 : pAngle == 90 ? FI_V : pAngle < 180 ? FI_Z2 : pAngle == 180 ? FI_H : FI_Z3;
        if (edgeFilter && pAngle != 90 && pAngle != 180) {
            F.corner = pAngle > 90 && pAngle < 180 && (w + h) >= 24;
            F.strA = F.hA ? edge_strength(w, h, smooth, pAngle - 90) : 0;
            F.strL = F.hL ? edge_strength(w, h, smooth, pAngle - 180) : 0;
            F.nA = imin(w, maxXd - x + 1) + (pAngle < 90 ? h : 0) + 1;
            F.nL = imin(h, maxYd - y + 1) + (pAngle > 180 ? w : 0) + 1;
            F.nUA = edge_upsample_used(w, h, smooth, pAngle - 90) ? w + (pAngle < 90 ? h : 0) : 0;
            F.nUL = edge_upsample_used(w, h, smooth, pAngle - 180) ? h + (pAngle > 180 ? w : 0) : 0;
        }
        if (pAngle < 90) F.dx = stab(av1r_dr_intra_derivative, pAngle);
        else if (pAngle > 90 && pAngle < 180) F.dx = stab(av1r_dr_intra_derivative, 180 - pAngle);
        if (pAngle > 90 && pAngle < 180) F.dy = stab(av1r_dr_intra_derivative, pAngle - 90);
        else if (pAngle > 180) F.dy = stab(av1r_dr_intra_derivative, 270 - pAngle);
    } else {
        F.cls = mode == AV1R_DC_PRED ? FI_DC : mode == AV1R_SMOOTH_PRED ? FI_SMOOTH : mode == AV1R_SMOOTH_V_PRED ? FI_SMOOTH_V
              : mode == AV1R_SMOOTH_H_PRED ? FI_SMOOTH_H : FI_PAETH;
    }
    return F;
}

// Sm_Weights_Tx_4x4 / 8x8 / 16x16 (the spec's table, av1r_sm_weights[0..28)) as dwords:
// weights 4d .. 4d + 3 of side 1 << log2 (<= 16) in dword d
DEV uint32_t fi_smw(int log2, int d)
{
    if (log2 == 2) return 0x405595ffu;                                  // 255 149 85 64
    if (log2 == 3) return d == 0 ? 0x6992c5ffu : 0x20253249u;           // 255 197 146 105 | 73 50 37 32
    return d == 0 ? 0xaac4e1ffu : d == 1 ? 0x54667b91u : d == 2 ? 0x212b3644u : 0x1011141au;
}

// sum over the lanes of each row of 16 (DPP shifts), returned from lane 15 of row r
DEV int fi_row_sum(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
    return v;
}

// After the dependency wait: gather, predict, add, store, publish (see the file comment).
// R: the residual quad of this lane (res_prefetch<64, 16>).  Ends with the stores issued.
// the wave-uniform value in a scalar register (the parameters cross the dependency wait,
// after which the compiler no longer knows them uniform: every table read or branch on them
// became a readfirstlane + scalar load of its own)
DEV int fi_uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// Intra_Edge_Kernel[strength - 1][j] (spec 7.11.2.12, av1r_edge_kernel): {0,4,8,4,0},
// {0,5,6,5,0}, {2,4,4,4,2} -- symmetric, as selects instead of table reads
DEV int fi_ek0(int str) { return str == 3 ? 2 : 0; }
DEV int fi_ek1(int str) { return str == 2 ? 5 : 4; }
DEV int fi_ek2(int str) { return str == 1 ? 8 : str == 2 ? 6 : 4; }

template <int MAX>
DEV void fi_run(const KParams& k, const WorkItem& tb, const FiParams& F0, TbLds<MAX>& L, const GranEdges& G, uint2 res,
    uint32_t epoch, bool gran)
{
    FiParams F;
    F.cls = fi_uni(F0.cls);
    F.log2W = fi_uni(F0.log2W);
    F.log2H = fi_uni(F0.log2H);
    F.hA = fi_uni(F0.hA) != 0;
    F.hL = fi_uni(F0.hL) != 0;
    F.cfl = fi_uni(F0.cfl) != 0;
    F.aboveLimit = fi_uni(F0.aboveLimit);
    F.leftLimit = fi_uni(F0.leftLimit);
    F.strA = fi_uni(F0.strA);
    F.strL = fi_uni(F0.strL);
    F.nA = fi_uni(F0.nA);
    F.nL = fi_uni(F0.nL);
    F.nUA = fi_uni(F0.nUA);
    F.nUL = fi_uni(F0.nUL);
    F.corner = fi_uni(F0.corner);
    F.dx = fi_uni(F0.dx);
    F.dy = fi_uni(F0.dy);
    F.alpha = fi_uni(F0.alpha);
    F.maxLW = fi_uni(F0.maxLW);
    F.maxLH = fi_uni(F0.maxLH);
    const int t = coop_lane<64>();
    const int plane = tb.plane, x = tb.x, y = tb.y;
    const int log2W = F.log2W, log2H = F.log2H, w = 1 << log2W, h = 1 << log2H;
    const DevPlane& dst = k.cur.pl[plane];
    IntraLds& I = L.intra;
    // CFL: the co-located luma of this lane's four pixels (flow read site: the block's luma,
    // written by earlier items -- sc1 loads after the dependency wait),
    // issued before the edge gather so that its loads overlap the granule polls
    const int nq = (w * h) >> 2;
    const int w4 = w >> 2;
    const int qi = t >> (log2W - 2), qj = (t & (w4 - 1)) << 2;  // this lane's quad: row, first column
    int cv[4] = {0, 0, 0, 0};
    int csum = 0;
    if (F.cfl) {
        const DevPlane& luma = k.cur.pl[0];
        const bool coh = G.coh;
        if (t < nq) {
            const int ly = imin((y + qi) << 1, F.maxLH - 2);
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int lx = imin((x + qj + b) << 1, F.maxLW - 2);
                const int v = ldp_c(luma, lx, ly, coh) + ldp_c(luma, lx + 1, ly, coh) + ldp_c(luma, lx, ly + 1, coh) +
                              ldp_c(luma, lx + 1, ly + 1, coh);
                cv[b] = v << 1;
                csum += cv[b];
            }
        }
    }
    gran_gather<64>(dst, plane, x, y, F.hL, F.hA, F.aboveLimit, F.leftLimit, I, G);
    coop_sync<64>();  // (wave level: the units are in LDS)
    trace_stamp(G.tr, 8);
    // raw AboveRow / LeftCol (coop_intra_edges' assembly, read in place from the units)
    const uint8_t* ta = I.tmp;
    const uint8_t* tl = I.tmp2;
    const int aLim = F.aboveLimit - x, lLim = F.leftLimit - y;
    // each edge value is one LDS byte at a uniformly chosen base and clamp, or a constant:
    // no branches, so every read of the pass goes out before the one wait
    const uint8_t* bA = F.hA ? ta : tl;  // (!hA: the left neighbour (x - 1, y) stands in)
    const uint8_t* bL = F.hL ? tl : ta;
    const int cA = F.hA ? aLim : 0, cL = F.hL ? lLim : 0;
    const int kA = F.hA || F.hL ? -1 : 127, kL = F.hA || F.hL ? -1 : 129;  // neither edge: constants
    auto rawA = [&](int i) -> int { const int v = bA[imin(cA, i)]; return kA >= 0 ? kA : v; };
    auto rawL = [&](int i) -> int { const int v = bL[imin(cL, i)]; return kL >= 0 ? kL : v; };
    const uint8_t* bC = F.hA && F.hL ? tl + 4 * 39 + 3 : F.hA ? ta : tl;
    const int c0 = *bC;
    const int corner0 = F.hA || F.hL ? c0 : 128;
    const int cs = F.corner ? r2(rawL(0) * 5 + corner0 * 6 + rawA(0) * 5, 4) : corner0;
    uint8_t* EA = I.above + EDGE_OFF;
    uint8_t* EL = I.left + EDGE_OFF;
    // the directional classes build AboveRow / LeftCol (edge filter, upsampling) in LDS;
    // the others (DC, V, H, smooth, Paeth: no filter, no upsampling) read the units directly
    const bool dirc = F.cls == FI_Z1 || F.cls == FI_Z2 || F.cls == FI_Z3;
    const uint8_t* A = EA;
    const uint8_t* Lc = EL;
    if (dirc) {
        // AboveRow / LeftCol in two passes with no per-tap branching: lane l writes the filter
        // input e[l] (e[0] the corner or its filtered value, e[k] = raw [k - 1]); where a side is
        // filtered, a second pass runs the 5-tap filter over e[] (clamped indices, plain LDS
        // reads) into AboveRow / LeftCol; where no side is, e[] already is them (EA = eA + 1)
        const bool filt = (F.strA | F.strL) != 0;
        uint8_t* eA = filt ? I.upA : EA - 1;
        uint8_t* eL = filt ? I.upL : EL - 1;
        if (t <= w + h) {
            eA[t] = (uint8_t)(t == 0 ? cs : rawA(t - 1));
            eL[t] = (uint8_t)(t == 0 ? cs : rawL(t - 1));
        }
        if (filt) {
            coop_sync<64>();
            if (t <= w + h) {
                int a = eA[t], l = eL[t];
                if (F.strA && t >= 1 && t < F.nA) {
                    const int n1 = F.nA - 1, k0 = fi_ek0(F.strA), k1 = fi_ek1(F.strA), k2 = fi_ek2(F.strA);
                    a = (k0 * (eA[imax(t - 2, 0)] + eA[imin(t + 2, n1)]) + k1 * (eA[t - 1] + eA[imin(t + 1, n1)]) + k2 * a + 8) >> 4;
                }
                if (F.strL && t >= 1 && t < F.nL) {
                    const int n1 = F.nL - 1, k0 = fi_ek0(F.strL), k1 = fi_ek1(F.strL), k2 = fi_ek2(F.strL);
                    l = (k0 * (eL[imax(t - 2, 0)] + eL[imin(t + 2, n1)]) + k1 * (eL[t - 1] + eL[imin(t + 1, n1)]) + k2 * l + 8) >> 4;
                }
                EA[t - 1] = (uint8_t)a;
                EL[t - 1] = (uint8_t)l;
            }
        }
        coop_sync<64>();
        trace_stamp(G.tr, 12);
        // upsampling: buf[2i - 1], buf[2i] from the edge (index -2 .. 2n - 2)
        if (F.nUA | F.nUL) {
#pragma unroll
            for (int side = 0; side < 2; side++) {
                const int n = side ? F.nUL : F.nUA;
                if (!n) continue;
                const uint8_t* e = side ? EL : EA;
                uint8_t* buf = (side ? I.upL : I.upA) + EDGE_OFF;
                if (t < n) {
                    const int d0 = t == 0 ? e[-1] : e[t - 2];
                    const int d1 = e[t - 1], d2 = e[t];
                    const int d3 = t + 1 <= n - 1 ? e[t + 1] : e[n - 1];
                    buf[2 * t - 1] = (uint8_t)clip1(r2(-d0 + 9 * d1 + 9 * d2 - d3, 4));
                    buf[2 * t] = (uint8_t)d2;
                }
                if (t == 0) buf[-2] = e[-1];
            }
            coop_sync<64>();
            if (F.nUA) A = I.upA + EDGE_OFF;
            if (F.nUL) Lc = I.upL + EDGE_OFF;
        }
    }
    // DC (and CFL's DC): the edge sums over lanes 0..15 (w, h <= 16)
    int dc = 128;
    if (F.cls == FI_DC) {
        int v = (F.hA && t < w ? rawA(t) : 0) + (F.hL && t < h ? rawL(t) : 0);
        const int s = __builtin_amdgcn_readlane(fi_row_sum(v), 15);
        if (F.hA && F.hL) {
            // (s + (w + h) / 2) / (w + h): a shift when square; otherwise w + h = 3 << k or
            // 5 << k (sides 4..16): the quotient from a float reciprocal, then corrected
            // by one either way (n < 2^14: exact within one ulp)
            const int n = s + ((w + h) >> 1);
            if (log2W == log2H) {
                dc = n >> (log2W + 1);
            } else {
                const int d = w + h;
                int q = (int)((float)n * __builtin_amdgcn_rcpf((float)d));
                q += (q + 1) * d <= n;
                q -= q * d > n;
                dc = q;
            }
        }
        else if (F.hL) dc = clip1((s + (h >> 1)) >> log2H);
        else if (F.hA) dc = clip1((s + (w >> 1)) >> log2W);
    }
    trace_stamp(G.tr, 13);
    // the prediction of this lane's quad
    uint32_t p = 0;
    if (t < nq) {
        const int i = qi;
        const int upA = F.nUA ? 1 : 0, upL = F.nUL ? 1 : 0;
        switch (F.cls) {
        case FI_DC: p = (uint32_t)dc * 0x01010101u; break;
        case FI_V: p = rawA(qj) | rawA(qj + 1) << 8 | rawA(qj + 2) << 16 | (uint32_t)rawA(qj + 3) << 24; break;
        case FI_H: p = (uint32_t)rawL(i) * 0x01010101u; break;
        case FI_Z1: {
            const int idx = (i + 1) * F.dx;
            const int shift = ((idx << upA) >> 1) & 0x1F;
            const int maxBaseX = (w + h - 1) << upA;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int base = (idx >> (6 - upA)) + ((qj + b) << upA);
                const int v = base < maxBaseX ? r2(A[base] * (32 - shift) + A[base + 1] * shift, 5) : A[maxBaseX];
                p |= (uint32_t)v << (8 * b);
            }
            break;
        }
        case FI_Z2: {
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int j = qj + b;
                int idx = (j << 6) - (i + 1) * F.dx;
                int base = idx >> (6 - upA);
                int v;
                if (base >= -(1 << upA)) {
                    const int shift = ((idx << upA) >> 1) & 0x1F;
                    v = r2(A[base] * (32 - shift) + A[base + 1] * shift, 5);
                } else {
                    idx = (i << 6) - (j + 1) * F.dy;
                    base = idx >> (6 - upL);
                    const int shift = ((idx << upL) >> 1) & 0x1F;
                    v = r2(Lc[base] * (32 - shift) + Lc[base + 1] * shift, 5);
                }
                p |= (uint32_t)v << (8 * b);
            }
            break;
        }
        case FI_Z3: {
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int idx = (qj + b + 1) * F.dy;
                const int base = (idx >> (6 - upL)) + (i << upL);
                const int shift = ((idx << upL) >> 1) & 0x1F;
                p |= (uint32_t)r2(Lc[base] * (32 - shift) + Lc[base + 1] * shift, 5) << (8 * b);
            }
            break;
        }
        case FI_PAETH: {
            const uint32_t a4 = rawA(qj) | rawA(qj + 1) << 8 | rawA(qj + 2) << 16 | (uint32_t)rawA(qj + 3) << 24;
            const int l = rawL(i), tl0 = corner0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int a = (a4 >> (8 * b)) & 0xff;
                const int base = a + l - tl0;
                const int pL = iabs(base - l), pT = iabs(base - a), pTL = iabs(base - tl0);
                p |= (uint32_t)((pL <= pT && pL <= pTL) ? l : (pT <= pTL ? a : tl0)) << (8 * b);
            }
            break;
        }
        default: {  // SMOOTH, SMOOTH_V, SMOOTH_H
            const uint32_t a4 = rawA(qj) | rawA(qj + 1) << 8 | rawA(qj + 2) << 16 | (uint32_t)rawA(qj + 3) << 24;
            const uint32_t wx4 = fi_smw(log2W, qj >> 2);
            const int wy = (fi_smw(log2H, i >> 2) >> (8 * (i & 3))) & 0xff;
            const int l = rawL(i), bl = rawL(h - 1), tr = rawA(w - 1);
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int a = (a4 >> (8 * b)) & 0xff, wx = (wx4 >> (8 * b)) & 0xff;
                int v;
                if (F.cls == FI_SMOOTH) v = r2(wy * a + (256 - wy) * bl + wx * l + (256 - wx) * tr, 9);
                else if (F.cls == FI_SMOOTH_V) v = r2(wy * a + (256 - wy) * bl, 8);
                else v = r2(wx * l + (256 - wx) * tr, 8);
                p |= (uint32_t)v << (8 * b);
            }
            break;
        }
        }
    }
    if (F.cfl) {
        // the luma average over the whole block (rows of 16 lanes, then across rows)
        const int rs = fi_row_sum(csum);
        const int s = __builtin_amdgcn_readlane(rs, 15) + __builtin_amdgcn_readlane(rs, 31) + __builtin_amdgcn_readlane(rs, 47) +
                      __builtin_amdgcn_readlane(rs, 63);
        const int avg = r2(s, log2W + log2H);
        uint32_t q = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) q |= (uint32_t)clip1(dc + r2s(F.alpha * (cv[b] - avg), 6)) << (8 * b);
        p = q;
    }
    trace_stamp(G.tr, 9);
    const uint32_t o = add4(p, res);
    // the granules first (what the next items wait for), then the frame
    if (gran) {
        // granules from the registers: the bottom row's units are the last row's quads; a
        // right-column unit is byte 3 of four vertically adjacent quads (the plane's granule
        // arrays from G, set up before the wait: no dependent parameter load here)
        const uint64_t tag = (uint64_t)epoch << 32;
        // the quads below in the same 16-lane DPP row (a publishing lane is the row's
        // lane w4 - 1 + 4 * w4 * k, so its three partners t + w4, + 2 w4, + 3 w4 stay in the row)
        uint32_t o1, o2, o3;
        if (w4 == 1) {
            o1 = __builtin_amdgcn_update_dpp(0, (int)o, 0x101, 0xf, 0xf, true);  // row_shl:1
            o2 = __builtin_amdgcn_update_dpp(0, (int)o, 0x102, 0xf, 0xf, true);
            o3 = __builtin_amdgcn_update_dpp(0, (int)o, 0x103, 0xf, 0xf, true);
        } else if (w4 == 2) {
            o1 = __builtin_amdgcn_update_dpp(0, (int)o, 0x102, 0xf, 0xf, true);
            o2 = __builtin_amdgcn_update_dpp(0, (int)o, 0x104, 0xf, 0xf, true);
            o3 = __builtin_amdgcn_update_dpp(0, (int)o, 0x106, 0xf, 0xf, true);
        } else {
            o1 = __builtin_amdgcn_update_dpp(0, (int)o, 0x104, 0xf, 0xf, true);
            o2 = __builtin_amdgcn_update_dpp(0, (int)o, 0x108, 0xf, 0xf, true);
            o3 = __builtin_amdgcn_update_dpp(0, (int)o, 0x10c, 0xf, 0xf, true);
        }
        if (t < nq && qi == h - 1)
            __hip_atomic_store(const_cast<uint64_t*>(G.h) + (size_t)((y + h - 1) >> 2) * G.gw + (x >> 2) + (qj >> 2), tag | o,
                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t < nq && qj == w - 4 && (qi & 3) == 0) {
            const uint32_t v = (o >> 24) | ((o1 >> 24) << 8) | ((o2 >> 24) << 16) | ((o3 >> 24) << 24);
            __hip_atomic_store(const_cast<uint64_t*>(G.v) + (size_t)((x + w - 1) >> 2) * G.gh + (y >> 2) + (qi >> 2), tag | v,
                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (t < nq) stp4_c(dst, x + qj, y + qi, o, G.coh);
}
