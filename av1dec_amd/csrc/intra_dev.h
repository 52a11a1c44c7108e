// intra_dev.h -- workgroup-cooperative intra prediction for gfx950.
//
// Restates Block::IntraPredict (decoder/IntraPredict.cpp:563-667) as a cooperative
// device routine: the edge arrays (AboveRow/LeftCol) are gathered by all lanes into
// LDS, the 5-tap edge filter and the 2x upsampler run one output per lane on a
// snapshot of the edge, and the predictors compute one pixel per lane.  Filter-intra's
// serial 4x2 recursion (:112-149) runs as an anti-diagonal wavefront.  Usable from
// group of NT cooperating lanes: a whole 256-lane workgroup or a single wave (NT = 64,
// several items per workgroup, wave-level synchronisation; see coop_sync in av1r_dev.h).
#pragma once
#include "av1r_dev.h"

#define EDGE_OFF 16
#define EDGE_LEN (EDGE_OFF + 144)

struct IntraLds {
    uint8_t above[EDGE_LEN];
    uint8_t left[EDGE_LEN];
    uint8_t tmp[EDGE_LEN];
    uint8_t tmp2[EDGE_LEN];
    uint8_t upA[EDGE_LEN];
    uint8_t upL[EDGE_LEN];
    int sum[2];
};

struct IntraParams {
    int plane, x, y, log2W, log2H;
    int haveLeft, haveAbove, haveAR, haveBL;
    int mode;          // PREDICTION_MODE (luma numbering); CFL handled by the caller
    int angleDelta;
    int filterIntra;   // plane 0 && use_filter_intra
    int filterIntraMode;
    int smooth;        // filterType: above/left neighbour uses a smooth mode
    int edgeFilter;    // enable_intra_edge_filter
};

DEV int edge_strength(int w, int h, int filterType, int delta)
{
    int d = iabs(delta), blkWh = w + h, s = 0;
    if (!filterType) {
        if (blkWh <= 8) {
            if (d >= 56) s = 1;
        } else if (blkWh <= 16) {
            if (d >= 40) s = 1;
        } else if (blkWh <= 24) {
            if (d >= 8) s = 1;
            if (d >= 16) s = 2;
            if (d >= 32) s = 3;
        } else if (blkWh <= 32) {
            s = 1;
            if (d >= 4) s = 2;
            if (d >= 32) s = 3;
        } else {
            s = 3;
        }
    } else {
        if (blkWh <= 8) {
            if (d >= 40) s = 1;
            if (d >= 64) s = 2;
        } else if (blkWh <= 16) {
            if (d >= 20) s = 1;
            if (d >= 48) s = 2;
        } else if (blkWh <= 24) {
            if (d >= 4) s = 3;
        } else {
            s = 3;
        }
    }
    return s;
}
DEV int edge_upsample_used(int w, int h, int filterType, int delta)
{
    int d = iabs(delta), blkWh = w + h;
    if (d <= 0 || d >= 40) return 0;
    return filterType ? (blkWh <= 8) : (blkWh <= 16);
}

// The TinyItem of an intra TB of at most 8x8 (av1r_dev.h; k_mi_zero writes it over the
// item's WorkItem): fi_setup's parameters (intra_fast.h, restating IntraPredict::predict_intra,
// IntraPredict.cpp:563-630, with the directional edge preparation :389-437), per lane (the
// tables through plain loads), plus the item's granule masks m[0..3] (m[3]: its residual tile,
// build_schedule's fourth mask word) and dependency list.
DEV TinyItem tiny_from_item(const KParams& k, const WorkItem& w, const DevBlock& blk, const uint32_t* m)
{
    const av1r_frame_hdr& hd = *k.hdr;
    const int plane = w.plane, sub = plane ? 1 : 0, x = w.x, y = w.y;
    const int log2W = av1r_tx_w_log2[w.tx_size], log2H = av1r_tx_h_log2[w.tx_size];
    const int tw = 1 << log2W, th = 1 << log2H;
    const int maxXd = (k.mi_cols * 4) >> sub, maxYd = (k.mi_rows * 4) >> sub;
    const bool hA = w.flags & AV1R_TB_HAVE_ABOVE, hL = w.flags & AV1R_TB_HAVE_LEFT;
    const int aboveLimit = imin(maxXd - 1, x + ((w.flags & AV1R_TB_HAVE_AR) ? 2 * tw : tw) - 1);
    const int leftLimit = imin(maxYd - 1, y + ((w.flags & AV1R_TB_HAVE_BL) ? 2 * th : th) - 1);
    const bool cfl = plane > 0 && blk.uv_mode == AV1R_UV_CFL_PRED;
    const int mode = plane == 0 ? blk.y_mode : (cfl ? AV1R_DC_PRED : blk.uv_mode);
    const int smooth = plane ? ((blk.flags & (AV1R_BLK_SMOOTH_A_UV | AV1R_BLK_SMOOTH_L_UV)) != 0)
                             : ((blk.flags & (AV1R_BLK_SMOOTH_A_Y | AV1R_BLK_SMOOTH_L_Y)) != 0);
    int cls, strA = 0, strL = 0, nA = 0, nL = 0, nUA = 0, nUL = 0, corner = 0, dx = 0, dy = 0;
    if (mode >= AV1R_V_PRED && mode <= AV1R_D67_PRED) {
        const int pAngle = av1r_mode_to_angle[mode] + (plane == 0 ? blk.angle_delta_y : blk.angle_delta_uv) * 3;
        cls = pAngle < 90 ? FI_Z1 : pAngle == 90 ? FI_V : pAngle < 180 ? FI_Z2 : pAngle == 180 ? FI_H : FI_Z3;
        if (hd.enable_intra_edge_filter && pAngle != 90 && pAngle != 180) {
            corner = pAngle > 90 && pAngle < 180 && (tw + th) >= 24;
            strA = hA ? edge_strength(tw, th, smooth, pAngle - 90) : 0;
            strL = hL ? edge_strength(tw, th, smooth, pAngle - 180) : 0;
            nA = imin(tw, maxXd - x + 1) + (pAngle < 90 ? th : 0) + 1;
            nL = imin(th, maxYd - y + 1) + (pAngle > 180 ? tw : 0) + 1;
            nUA = edge_upsample_used(tw, th, smooth, pAngle - 90) ? tw + (pAngle < 90 ? th : 0) : 0;
            nUL = edge_upsample_used(tw, th, smooth, pAngle - 180) ? th + (pAngle > 180 ? tw : 0) : 0;
        }
        if (pAngle < 90) dx = av1r_dr_intra_derivative[pAngle];
        else if (pAngle > 90 && pAngle < 180) dx = av1r_dr_intra_derivative[180 - pAngle];
        if (pAngle > 90 && pAngle < 180) dy = av1r_dr_intra_derivative[pAngle - 90];
        else if (pAngle > 180) dy = av1r_dr_intra_derivative[270 - pAngle];
    } else {
        cls = mode == AV1R_DC_PRED ? FI_DC : mode == AV1R_SMOOTH_PRED ? FI_SMOOTH : mode == AV1R_SMOOTH_V_PRED ? FI_SMOOTH_V
            : mode == AV1R_SMOOTH_H_PRED ? FI_SMOOTH_H : FI_PAETH;
    }
    TinyItem r;
    r.x = (uint16_t)x;
    r.y = (uint16_t)y;
    r.shape = (uint8_t)(plane | (log2W - 2) << 2 | (log2H - 2) << 3 | cls << 4);
    r.flags = (uint8_t)((hA ? TI_HA : 0u) | (hL ? TI_HL : 0u) | (cfl ? TI_CFL : 0u) | (corner ? TI_CORNER : 0u) | ((w.pub & 1) ? TI_PUB : 0u));
    r.str = (uint8_t)(strA | strL << 4);
    r.lim = (uint8_t)((aboveLimit - x) | (leftLimit - y) << 4);
    r.nA = (uint8_t)nA, r.nL = (uint8_t)nL, r.nUA = (uint8_t)nUA, r.nUL = (uint8_t)nUL;
    r.masks = (uint8_t)((m[0] & 15) | (m[2] & 15) << 4);
    r.mC = (uint8_t)(m[1] & 3);
    r.p0 = (uint16_t)(cfl ? blk.max_luma_w : dx);
    r.p1 = (uint16_t)(cfl ? blk.max_luma_h : dy);
    r.alpha = (int8_t)(cfl ? (plane == 1 ? blk.cfl_alpha_u : blk.cfl_alpha_v) : 0);
    r.pad = 0;
    r.dep_off = w.dep_off;
    r.dep_cnt = w.dep_cnt;
    r.zero = 0;
    r.res = m[3];
    return r;
}

// The edge preparation of directionalIntraPredict (IntraPredict.cpp:394-437) for both
// edges at once, three barriers in all: the corner filter (filterCorner, :204-209) folded
// into the copy pass, both intraEdgeFilter passes (:324-337) in one, both upsamples
// (:354-370) in one.  nA / nL: filter lengths (numPx), strA / strL: strengths (0: none),
// nUA / nUL: upsampled lengths (0: no upsampling).
template <int NT>
DEV void coop_edge_prepare(uint8_t* above, uint8_t* left, IntraLds& L, bool corner, int strA, int nA, int strL,
    int nL, int nUA, int nUL, unsigned long long* tr = nullptr)
{
    const int t = coop_lane<NT>(), nt = NT;
    const int cs = corner ? r2(left[0] * 5 + above[-1] * 6 + above[0] * 5, 4) : above[-1];
    int kA[5], kL[5];  // the two filters' taps (uniform: scalar loads)
#pragma unroll
    for (int j = 0; j < 5; j++) {
        kA[j] = strA ? ctab<NT>(av1r_edge_kernel[strA - 1], j) : 0;
        kL[j] = strL ? ctab<NT>(av1r_edge_kernel[strL - 1], j) : 0;
    }
    if (strA)
        for (int i = t; i < nA; i += nt) L.tmp[i] = i == 0 ? (uint8_t)cs : above[i - 1];
    if (strL)
        for (int i = t; i < nL; i += nt) L.tmp2[i] = i == 0 ? (uint8_t)cs : left[i - 1];
    if (strA || strL || corner) coop_sync<NT>();
    trace_stamp(tr, 13);
    if (strA)
        for (int i = 1 + t; i < nA; i += nt) {
            int s = 0;
#pragma unroll
            for (int j = 0; j < 5; j++) s += kA[j] * L.tmp[CLIP3(0, nA - 1, i - 2 + j)];
            above[i - 1] = (uint8_t)((s + 8) >> 4);
        }
    if (strL)
        for (int i = 1 + t; i < nL; i += nt) {
            int s = 0;
#pragma unroll
            for (int j = 0; j < 5; j++) s += kL[j] * L.tmp2[CLIP3(0, nL - 1, i - 2 + j)];
            left[i - 1] = (uint8_t)((s + 8) >> 4);
        }
    if (corner && t == 0) {
        above[-1] = (uint8_t)cs;
        left[-1] = (uint8_t)cs;
    }
    if (strA || strL || corner) coop_sync<NT>();
    // upsampled buffers: index -2 .. 2 * numPx - 2 at up + EDGE_OFF; dup[k] = k == 0 ? e[-1]
    // : k <= numPx + 1 ? e[k - 2] : e[numPx - 1]
    for (int side = 0; side < 2; side++) {
        const int n = side ? nUL : nUA;
        if (!n) continue;
        const uint8_t* e = side ? left : above;
        uint8_t* buf = (side ? L.upL : L.upA) + EDGE_OFF;
        for (int i = t; i < n; i += nt) {
            int d0 = i == 0 ? e[-1] : e[i - 2];
            int d1 = e[i - 1];
            int d2 = e[i];
            int d3 = (i + 1 <= n - 1) ? e[i + 1] : e[n - 1];
            int s = -d0 + 9 * d1 + 9 * d2 - d3;
            buf[2 * i - 1] = (uint8_t)clip1(r2(s, 4));
            buf[2 * i] = (uint8_t)d2;
        }
        if (t == 0) buf[-2] = e[-1];
    }
    if (nUA || nUL) coop_sync<NT>();
}

DEV const uint8_t* sm_weights(int log2) { return av1r_sm_weights + ((1 << log2) - 4); }

// Gathers AboveRow / LeftCol (IntraPredict.cpp:571-611) of a (1<<log2W) x (1<<log2H)
// prediction at (x, y) of plane `plane` into L (global loads only; the caller issues the
// barrier before the edges are read, so independent loads can be overlapped with it).
template <int NT, bool COH>
DEV void coop_intra_edges(int miCols, int miRows, const DevPlane& src, int plane, int x, int y, int log2W,
    int log2H, bool hL, bool hA, bool hAR, bool hBL, IntraLds& L)
{
    const int t = coop_lane<NT>(), nt = NT;
    const int w = 1 << log2W, h = 1 << log2H;
    // predict_intra uses subsampling_x for both axes (IntraPredict.cpp:566-567)
    const int sub = plane ? 1 : 0;
    const int maxX = ((miCols * 4) >> sub) - 1;
    const int maxY = ((miRows * 4) >> sub) - 1;
    uint8_t* above = L.above + EDGE_OFF;
    uint8_t* left = L.left + EDGE_OFF;
    const int n = w + h;
    const int aboveLimit = imin(maxX, x + (hAR ? 2 * w : w) - 1);
    const int leftLimit = imin(maxY, y + (hBL ? 2 * h : h) - 1);
    // (flow read site, COH = true in k_flow: sc1 loads after the dependency-flag wait)
    for (int i = t; i < n; i += nt) {
        uint8_t a, l;
        if (!hA && hL) a = ldp<COH>(src, x - 1, y);
        else if (!hA && !hL) a = 127;
        else a = ldp<COH>(src, imin(aboveLimit, x + i), y - 1);
        if (!hL && hA) l = ldp<COH>(src, x, y - 1);
        else if (!hA && !hL) l = 129;
        else l = ldp<COH>(src, x - 1, imin(leftLimit, y + i));
        above[i] = a;
        left[i] = l;
    }
    if (t == 0) {
        uint8_t c;
        if (hA && hL) c = ldp<COH>(src, x - 1, y - 1);
        else if (hA) c = ldp<COH>(src, x, y - 1);
        else if (hL) c = ldp<COH>(src, x - 1, y);
        else c = 128;
        above[-1] = c;
        left[-1] = c;
    }
}

// k_flow's edge gather through granules (KParams::gran_h / gran_v).  The above run is the
// units of row (y-1)/4 from x/4 to aboveLimit/4, the left run the units of column (x-1)/4
// from y/4 to leftLimit/4, plus the corner pixel (x-1, y-1): exactly the pixels
// coop_intra_edges reads.  mask[0] (above) and mask[2] (left) flag, bit u = unit u of the
// run, the units written by an item of this launch; mask[1] bit 0 the corner's, bit 1 its
// granule (byte 3) is its owner's right column instead of its bottom row.  One lane per
// such unit re-reads its granule (sc1) until the tag is the launch's epoch, so the pixels
// arrive with the signal (no dependency flag, no second round trip).  The other units
// were final before the launch and are read from the frame.  The runs are staged in
// L.tmp / L.tmp2, then AboveRow / LeftCol are assembled as in coop_intra_edges.  Bounded:
// a spin gives up after ~1 s (or once another wave has) and sets the launch's error word.
// (LDS address-space pointers: through a generic pointer an LDS access is a flat_
// instruction, which also waits for the wave's outstanding global stores)
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

struct GranEdges {
    const uint32_t* mask;  // 4 words: above, corner, left, (unused)
    uint32_t mA, mC, mL;   // mask[0..2], loaded by the caller (k_flow: before its dependency wait)
    const uint64_t* h;     // this plane's gran_h / gran_v, gw units per row / gh per column
    const uint64_t* v;
    int gw, gh;
    uint32_t epoch;
    uint32_t* ctl;         // k_flow control block (FLOW_ERR)
    unsigned long long* tr;  // -DAV1R_TRACE timeline row (or null)
    bool coh;              // units read from the frame: sc1 or plain
};
// The gather half: the above run's units into L.tmp (pixel (x + i, y - 1) at byte i), the
// left run's into L.tmp2 (pixel (x - 1, y + i) at byte i), the corner's unit at L.tmp2
// word 39 (the pixel in its byte 3).  aboveLimit / leftLimit: as coop_intra_edges.
template <int NT>
DEV void gran_gather(const DevPlane& src, int plane, int x, int y, bool hL, bool hA, int aboveLimit, int leftLimit,
    IntraLds& L, const GranEdges& G)
{
    const int t = coop_lane<NT>();
    const int na = hA ? (aboveLimit >> 2) - (x >> 2) + 1 : 0;
    const int nl = hL ? (leftLimit >> 2) - (y >> 2) + 1 : 0;
    const int nq = na + nl + (hA && hL ? 1 : 0);
    uint32_t* stA = reinterpret_cast<uint32_t*>(L.tmp);
    uint32_t* stL = reinterpret_cast<uint32_t*>(L.tmp2);  // [39]: the corner's unit
    if ((NT == 64 || t < 64) && nq > 0) {
        const int lane = t & 63;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t spins = 0, lim = 0;
        bool dead = false;
        for (int base = 0; base < nq; base += 64) {
            const int q = base + lane;
            const bool act = q < nq;
            const int kind = q < na ? 0 : q < na + nl ? 1 : 2;  // above, left, corner
            const int u = kind == 0 ? q : q - na;
            const uint32_t cm = G.mC;
            const bool inl = act && (kind == 0 ? ((G.mA >> (u & 31)) & 1)
                                   : kind == 1 ? ((G.mL >> (u & 31)) & 1) : (cm & 1));
            const uint64_t* g = kind == 0 ? G.h + (size_t)((y - 1) >> 2) * G.gw + (x >> 2) + u
                              : kind == 1 ? G.v + (size_t)((x - 1) >> 2) * G.gh + (y >> 2) + u
                              : (cm & 2) ? G.v + (size_t)((x - 1) >> 2) * G.gh + ((y - 1) >> 2)
                                         : G.h + (size_t)((y - 1) >> 2) * G.gw + ((x - 1) >> 2);
            uint32_t val = 0;
            // (flow read site: in-launch units of other items are granules (inl); the frame is
            // read only for pixels final before the launch)
            if (act && !inl) {  // final before this launch
                const bool c = G.coh;
                if (kind == 0) {
                    val = ldp4_c(src, x + 4 * u, y - 1, c);
                } else if (kind == 1) {
                    const int py = y + 4 * u;
                    val = ldp_c(src, x - 1, py, c) | (ldp_c(src, x - 1, py + 1, c) << 8) |
                          (ldp_c(src, x - 1, py + 2, c) << 16) | ((uint32_t)ldp_c(src, x - 1, py + 3, c) << 24);
                } else {
                    val = (uint32_t)ldp_c(src, x - 1, y - 1, c) << 24;
                }
            }
            for (;;) {
                bool ok = true;
                if (inl && !dead) {
                    const uint64_t gv = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = (uint32_t)(gv >> 32) == G.epoch;
                    val = (uint32_t)gv;
                }
                if (__all(ok)) break;
                // (the launch's error word every AV1R_ERR_POLL_MASK + 1 spins: every spinning
                // wave of the chip polls this one line)
                const bool other =
                    (spins & AV1R_ERR_POLL_MASK) == 0 && __hip_atomic_load(G.ctl + FLOW_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                if (!lim) lim = flow_spin_limit(G.ctl);
                if (other || ++spins > lim || __builtin_amdgcn_s_memrealtime() - t0 > FLOW_WALL) {
                    if (lane == 0 && !other) {  // 2: an edge granule wait (1: a dependency flag wait)
                        __hip_atomic_store(G.ctl + FLOW_ERR, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(reinterpret_cast<uint32_t*>(*reinterpret_cast<uint32_t* const*>(G.ctl + FLOW_HOSTERR)),
                            2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    dead = true;
                    break;
                }
#ifndef AV1R_POLL_BACKOFF
#define AV1R_POLL_BACKOFF 8  // after this many polls a waiting wave sleeps 4x longer between polls (0: never); key frame -1 %
#endif
                if (AV1R_POLL_BACKOFF && spins > AV1R_POLL_BACKOFF) __builtin_amdgcn_s_sleep(4);
                else __builtin_amdgcn_s_sleep(1);
            }
            if (act) (kind == 0 ? stA + u : kind == 1 ? stL + u : stL + 39)[0] = val;
        }
    }
    trace_stamp(G.tr, 11);
}
template <int NT>
DEV void coop_intra_edges_gran(int miCols, int miRows, const DevPlane& src, int plane, int x, int y, int log2W,
    int log2H, bool hL, bool hA, bool hAR, bool hBL, IntraLds& L, const GranEdges& G)
{
    const int t = coop_lane<NT>();
    const int w = 1 << log2W, h = 1 << log2H;
    const int sub = plane ? 1 : 0;
    const int maxX = ((miCols * 4) >> sub) - 1;
    const int maxY = ((miRows * 4) >> sub) - 1;
    const int aboveLimit = imin(maxX, x + (hAR ? 2 * w : w) - 1);
    const int leftLimit = imin(maxY, y + (hBL ? 2 * h : h) - 1);
    gran_gather<NT>(src, plane, x, y, hL, hA, aboveLimit, leftLimit, L, G);
    coop_sync<NT>();
    const uint8_t* sa = L.tmp - x;   // pixel (px, y - 1) at sa[px]
    const uint8_t* sl = L.tmp2 - y;  // pixel (x - 1, py) at sl[py]
    uint8_t* above = L.above + EDGE_OFF;
    uint8_t* left = L.left + EDGE_OFF;
    for (int i = t; i < w + h; i += NT) {
        uint8_t a, l;
        if (!hA && hL) a = sl[y];
        else if (!hA && !hL) a = 127;
        else a = sa[imin(aboveLimit, x + i)];
        if (!hL && hA) l = sa[x];
        else if (!hA && !hL) l = 129;
        else l = sl[imin(leftLimit, y + i)];
        above[i] = a;
        left[i] = l;
    }
    if (t == 0) {
        uint8_t c;
        if (hA && hL) c = L.tmp2[4 * 39 + 3];
        else if (hA) c = sa[x];
        else if (hL) c = sl[y];
        else c = 128;
        above[-1] = c;
        left[-1] = c;
    }
}

// k_flow producer side of the granules: the bottom row and right column of a w x h region
// at (x, y) whose final pixels are in `px` (row stride ps), one granule per 4x4 unit.
// Follows the region's pixel stores; the caller's coop_sync must separate `px`'s writes.
template <int NT>
DEV void coop_publish_gran(const uint8_t* px, int ps, int x, int y, int w, int h, uint64_t* gh, uint64_t* gv, int gw,
    int ghn, uint32_t epoch)
{
    const int t = coop_lane<NT>();
    const int nw = w >> 2, nh = h >> 2;
    const uint64_t tag = (uint64_t)epoch << 32;
    for (int q = t; q < nw + nh; q += NT) {
        uint32_t v;
        uint64_t* g;
        if (q < nw) {
            v = *reinterpret_cast<const uint32_t*>(px + (h - 1) * ps + 4 * q);
            g = gh + (size_t)((y + h - 1) >> 2) * gw + (x >> 2) + q;
        } else {
            const int r = 4 * (q - nw);
            const uint8_t* c = px + r * ps + w - 1;
            v = c[0] | (c[ps] << 8) | (c[2 * ps] << 16) | ((uint32_t)c[3 * ps] << 24);
            g = gv + (size_t)((x + w - 1) >> 2) * ghn + (y >> 2) + (q - nw);
        }
        __hip_atomic_store(g, tag | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Predicts the (1<<log2W) x (1<<log2H) block into pred (row stride ps) from edges already
// gathered into L (coop_intra_edges + a barrier).  Ends with a coop_sync.
template <int NT>
DEV void coop_intra_from_edges(int miCols, int miRows, const IntraParams& P, IntraLds& L, uint8_t* pred, int ps,
    unsigned long long* tr = nullptr)
{
    const int t = coop_lane<NT>(), nt = NT;
    const int w = 1 << P.log2W, h = 1 << P.log2H;
    const int plane = P.plane, x = P.x, y = P.y;
    const int sub = plane ? 1 : 0;
    uint8_t* above = L.above + EDGE_OFF;
    uint8_t* left = L.left + EDGE_OFF;
    if (P.filterIntra) {
        // recursiveIntraPrediction (IntraPredict.cpp:112-149): cell (i2, j4) needs cells
        // (i2-1, j4-1..j4) and (i2, j4-1): process anti-diagonals d = i2 + j4.
        const int w4 = w >> 2, h2 = h >> 1;
        const int8_t* taps = av1r_filter_intra_taps + P.filterIntraMode * 56;
        for (int d = 0; d < w4 + h2 - 1; d++) {
            int i2lo = imax(0, d - (w4 - 1)), i2hi = imin(h2 - 1, d);
            int ncell = i2hi - i2lo + 1;
            for (int q = t; q < ncell * 8; q += nt) {
                int i2 = i2lo + (q >> 3), j4 = d - i2;
                int o = q & 7, i1 = o >> 2, j1 = o & 3;
                int p[7];
#pragma unroll
                for (int i = 0; i < 5; i++) {
                    if (!i2) p[i] = above[(j4 << 2) + i - 1];
                    else if (!j4 && !i) p[i] = left[(i2 << 1) - 1];
                    else p[i] = pred[((i2 << 1) - 1) * ps + (j4 << 2) + i - 1];
                }
#pragma unroll
                for (int i = 5; i < 7; i++) {
                    if (!j4) p[i] = left[(i2 << 1) + i - 5];
                    else p[i] = pred[((i2 << 1) + i - 5) * ps + (j4 << 2) - 1];
                }
                int pr = 0;
#pragma unroll
                for (int i = 0; i < 7; i++) pr += taps[((i1 << 2) + j1) * 7 + i] * p[i];
                // all reads of this diagonal complete before any write (next barrier)
                L.tmp[q] = (uint8_t)clip1(r2s(pr, 4));
            }
            coop_sync<NT>();
            for (int q = t; q < ncell * 8; q += nt) {
                int i2 = i2lo + (q >> 3), j4 = d - i2;
                int o = q & 7;
                pred[((i2 << 1) + (o >> 2)) * ps + (j4 << 2) + (o & 3)] = L.tmp[q];
            }
            coop_sync<NT>();
        }
        return;
    }

    const int mode = P.mode;
    if (mode >= AV1R_V_PRED && mode <= AV1R_D67_PRED) {
        // directionalIntraPredict (IntraPredict.cpp:379-483)
        const int maxXd = (miCols * 4) >> sub;
        const int maxYd = (miRows * 4) >> sub;  // subsampling_y == subsampling_x (4:2:0)
        int pAngle = ctab<NT>(av1r_mode_to_angle, mode) + P.angleDelta * 3;
        int upA = 0, upL = 0;
        const uint8_t* A = above;
        const uint8_t* Lc = left;
        if (P.edgeFilter && pAngle != 90 && pAngle != 180) {
            const bool corner = pAngle > 90 && pAngle < 180 && (w + h) >= 24;
            const int strA = P.haveAbove ? edge_strength(w, h, P.smooth, pAngle - 90) : 0;
            const int strL = P.haveLeft ? edge_strength(w, h, P.smooth, pAngle - 180) : 0;
            const int nA = imin(w, maxXd - x + 1) + (pAngle < 90 ? h : 0) + 1;
            const int nL = imin(h, maxYd - y + 1) + (pAngle > 180 ? w : 0) + 1;
            upA = edge_upsample_used(w, h, P.smooth, pAngle - 90);
            upL = edge_upsample_used(w, h, P.smooth, pAngle - 180);
            coop_edge_prepare<NT>(above, left, L, corner, strA, nA, strL, nL, upA ? w + (pAngle < 90 ? h : 0) : 0,
                upL ? h + (pAngle > 180 ? w : 0) : 0, tr);
            if (upA) A = L.upA + EDGE_OFF;
            if (upL) Lc = L.upL + EDGE_OFF;
        }
        trace_stamp(tr, 12);
        int dx = 0, dy = 0;
        if (pAngle < 90) dx = ctab<NT>(av1r_dr_intra_derivative, pAngle);
        else if (pAngle > 90 && pAngle < 180) dx = ctab<NT>(av1r_dr_intra_derivative, 180 - pAngle);
        if (pAngle > 90 && pAngle < 180) dy = ctab<NT>(av1r_dr_intra_derivative, pAngle - 90);
        else if (pAngle > 180) dy = ctab<NT>(av1r_dr_intra_derivative, 270 - pAngle);
        for (int q = t; q < w * h; q += nt) {
            int i = q >> P.log2W, j = q & (w - 1);
            int v;
            if (pAngle < 90) {
                int idx = (i + 1) * dx;
                int base = (idx >> (6 - upA)) + (j << upA);
                int shift = ((idx << upA) >> 1) & 0x1F;
                int maxBaseX = (w + h - 1) << upA;
                v = base < maxBaseX ? r2(A[base] * (32 - shift) + A[base + 1] * shift, 5) : A[maxBaseX];
            } else if (pAngle > 90 && pAngle < 180) {
                int idx = (j << 6) - (i + 1) * dx;
                int base = idx >> (6 - upA);
                if (base >= -(1 << upA)) {
                    int shift = ((idx << upA) >> 1) & 0x1F;
                    v = r2(A[base] * (32 - shift) + A[base + 1] * shift, 5);
                } else {
                    idx = (i << 6) - (j + 1) * dy;
                    base = idx >> (6 - upL);
                    int shift = ((idx << upL) >> 1) & 0x1F;
                    v = r2(Lc[base] * (32 - shift) + Lc[base + 1] * shift, 5);
                }
            } else if (pAngle > 180) {
                int idx = (j + 1) * dy;
                int base = (idx >> (6 - upL)) + (i << upL);
                int shift = ((idx << upL) >> 1) & 0x1F;
                v = r2(Lc[base] * (32 - shift) + Lc[base + 1] * shift, 5);
            } else if (pAngle == 90) {
                v = A[j];
            } else {
                v = Lc[i];
            }
            pred[i * ps + j] = (uint8_t)v;
        }
    } else if (mode == AV1R_DC_PRED) {
        // dcPredict (IntraPredict.cpp:485-508): wave-level sums
        int s = 0;
        if (t < 64) {
            if (P.haveAbove)
                for (int j = t; j < w; j += 64) s += above[j];
            if (P.haveLeft)
                for (int i = t; i < h; i += 64) s += left[i];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
            if (t == 0) L.sum[0] = s;
        }
        coop_sync<NT>();
        s = L.sum[0];
        int avg;
        if (P.haveLeft && P.haveAbove) avg = (s + ((w + h) >> 1)) / (w + h);
        else if (P.haveLeft) avg = clip1((s + (h >> 1)) >> P.log2H);
        else if (P.haveAbove) avg = clip1((s + (w >> 1)) >> P.log2W);
        else avg = 128;
        for (int q = t; q < w * h; q += nt) pred[(q >> P.log2W) * ps + (q & (w - 1))] = (uint8_t)avg;
    } else {
        const uint8_t* wx = sm_weights(P.log2W);
        const uint8_t* wy = sm_weights(P.log2H);
        for (int q = t; q < w * h; q += nt) {
            int i = q >> P.log2W, j = q & (w - 1);
            int v;
            if (mode == AV1R_PAETH_PRED) {
                // paethPredict (IntraPredict.cpp:151-171)
                int base = above[j] + left[i] - above[-1];
                int pL = iabs(base - left[i]), pT = iabs(base - above[j]), pTL = iabs(base - above[-1]);
                v = (pL <= pT && pL <= pTL) ? left[i] : (pT <= pTL ? above[j] : above[-1]);
            } else if (mode == AV1R_SMOOTH_PRED) {
                v = r2(wy[i] * above[j] + (256 - wy[i]) * left[h - 1] + wx[j] * left[i] + (256 - wx[j]) * above[w - 1], 9);
            } else if (mode == AV1R_SMOOTH_V_PRED) {
                v = r2(wy[i] * above[j] + (256 - wy[i]) * left[h - 1], 8);
            } else {  // SMOOTH_H_PRED
                v = r2(wx[j] * left[i] + (256 - wx[j]) * above[w - 1], 8);
            }
            pred[i * ps + j] = (uint8_t)v;
        }
    }
    coop_sync<NT>();
}

// Gather + predict (IntraPredict::predict_intra, IntraPredict.cpp:563-630).  Ends with a
// coop_sync.
template <int NT, bool COH>
DEV void coop_intra_predict(int miCols, int miRows, const DevPlane& src, const IntraParams& P,
    IntraLds& L, uint8_t* pred, int ps)
{
    coop_intra_edges<NT, COH>(miCols, miRows, src, P.plane, P.x, P.y, P.log2W, P.log2H, P.haveLeft, P.haveAbove, P.haveAR,
        P.haveBL, L);
    coop_sync<NT>();
    coop_intra_from_edges<NT>(miCols, miRows, P, L, pred, ps);
}
