// recon.hip -- block reconstruction kernels for gfx950.
//
//   k_level  one 64-lane workgroup per work item of a dependency level.  Transform
//            block items:
//            intra / palette / CFL prediction (or the already-predicted inter pixels),
//            dequantisation, 2-D inverse transform (rows then columns, one lane per
//            row/column, T[] in VGPRs), flip, add, clip, store.
//            Restates TransformBlock::decode/reconstruct/inverseTransform
//            (decoder/TransformBlock.cpp:2173-2456).
//            Inter items (one <= 32x32 tile of a block): Block::compute_prediction
//            (decoder/Block.cpp:100-174) -> InterPredict::predict_inter
//            (decoder/InterPredict.cpp:962-1049): 8-tap sub-pel convolve or warp per
//            reference, compound average / distance / wedge / difference-weighted /
//            inter-intra blends, OBMC, assembled per plane in an LDS tile.
//            Inter-intra items: the intra half of an inter-intra block, blended in place.
// The host (av1r_host.cpp) orders launches by dependency level so every pixel a work
// item reads was finalised by an earlier launch.
#include "av1r_dev.h"
#include "intra_dev.h"
#include "txfm_dev.h"

// ---------------------------------------------------------------------------------
// Transform blocks
// ---------------------------------------------------------------------------------
// LDS of one transform block of at most MAX x MAX samples.  The residual tile's row stride
// RS = MAX + 2 int16 is an odd number of dwords: rows and columns are bank-conflict free.
template <int MAX>
struct TbLds {
    static constexpr int RS = MAX + 2;
    static constexpr int CM = MAX > 32 ? 32 : MAX;  // largest chroma (CFL) transform side
    int16_t res[MAX * RS];  // the final residual, flips applied (tb_residual)
    uint8_t pred[MAX * MAX];
    int16_t cfl[CM * CM];   // CFL: the averaged co-located luma
    IntraLds intra;
    int sum;
};

template <int n>
DEV void row_pass(int16_t* row, int w, int kind, int rectScale, int rowShift, int lossless)
{
    int T[1 << n];
#pragma unroll
    for (int j = 0; j < (1 << n); j++) T[j] = (j < 32) ? row[j] : 0;
    if (rectScale) {
#pragma unroll
        for (int j = 0; j < (1 << n); j++) T[j] = tx::rnd12(T[j] * 2896);
    }
    tx::run1d<n>(T, lossless ? 3 : kind, 16, 2);
#pragma unroll
    for (int j = 0; j < (1 << n); j++) row[j] = (int16_t)CLIP3(-32768, 32767, r2(T[j], rowShift));
}
// Column pass of one column, written back as the final residual of output column `out`
// (the left-right flip), rows flipped if flipUD.  Only ever one wave runs it (w <= 64), and
// a wave's LDS accesses complete in order, so every lane has read its column before any
// lane overwrites one.  The residual is saturated to int16: clip1(pred + r) is unchanged
// by that for any 8-bit prediction.
template <int n, int RS>
DEV void col_pass(const int16_t* col, int16_t* out, int kind, int colShift, int lossless, int flipUD)
{
    int T[1 << n];
#pragma unroll
    for (int i = 0; i < (1 << n); i++) T[i] = col[i * RS];
    tx::run1d<n>(T, lossless ? 3 : kind, 16, 0);
#pragma unroll
    for (int yy = 0; yy < (1 << n); yy++) {
        const int i = flipUD ? (1 << n) - 1 - yy : yy;
        out[i * RS] = (int16_t)CLIP3(-32768, 32767, r2(T[yy], colShift));
    }
}

// reconstruct() + inverseTransform() (TransformBlock.cpp:2173-2276) into L.res, flips
// applied.  Reads only the batch (coefficients, block record), never the frame: the
// dataflow kernel runs it before the item's dependencies are complete.  c0: the lane's
// first coefficient, prefetched by the caller.  Ends with a coop_sync.
template <int NT, int MAX, class TB>
DEV void tb_residual(const KParams& k, const TB& tb, const DevBlock& blk, int16_t* res, uint32_t c0)
{
    constexpr int RS = MAX + 2;
    const int t = coop_lane<NT>();
    const int txSz = tb.tx_size;
    const int w = av1r_tx_w[txSz], h = av1r_tx_h[txSz];
    const int log2W = av1r_tx_w_log2[txSz], log2H = av1r_tx_h_log2[txSz];
    const int tw = imin(w, 32), th = imin(h, 32), ltw = imin(log2W, 5);
    const av1r_frame_hdr& hd = *k.hdr;
    for (int q = t; q < th * w; q += NT) res[(q >> log2W) * RS + (q & (w - 1))] = 0;
    coop_sync<NT>();
    int dqDenom = 1;
    if (txSz == AV1R_TX_32X32 || txSz == AV1R_TX_16X32 || txSz == AV1R_TX_32X16 || txSz == AV1R_TX_16X64 || txSz == AV1R_TX_64X16)
        dqDenom = 2;
    else if (txSz == AV1R_TX_64X64 || txSz == AV1R_TX_32X64 || txSz == AV1R_TX_64X32)
        dqDenom = 4;
    const int plane = tb.plane;
    const int dcDelta = plane == 0 ? hd.delta_q_y_dc : plane == 1 ? hd.delta_q_u_dc : hd.delta_q_v_dc;
    const int acDelta = plane == 0 ? 0 : plane == 1 ? hd.delta_q_u_ac : hd.delta_q_v_ac;
    const int dcQ = av1r_dc_qlookup[CLIP3(0, 255, blk.qindex + dcDelta)];
    const int acQ = av1r_ac_qlookup[CLIP3(0, 255, blk.qindex + acDelta)];
    for (int q = t; q < tb.coef_cnt; q += NT) {
        const uint32_t c = q == t ? c0 : coef_at(k, tb.coef_off, tb.flags, q);  // the first NT were prefetched by the caller
        int pos = AV1R_COEF_POS(c), level = AV1R_COEF_LEVEL(c);
        int d = (int)((uint32_t)level * (uint32_t)(pos == 0 ? dcQ : acQ));
        int sign = d < 0 ? -1 : 1;
        int d2 = sign * (iabs(d) & 0xffffff) / dqDenom;
        res[(pos >> ltw) * RS + (pos & (tw - 1))] = (int16_t)CLIP3(-(1 << 15), (1 << 15) - 1, d2);
    }
    coop_sync<NT>();
    const int lossless = (blk.flags & AV1R_BLK_LOSSLESS) != 0;
    const int type = tb.tx_type;
    const int rowShift = lossless ? 0 : av1r_tx_row_shift[txSz];
    const int colShift = lossless ? 0 : 4;
    const int rect = iabs(log2W - log2H) == 1;
    const int rk = tx::row_kind(type), ck = tx::col_kind(type);
    // rows >= 32 of a 64-high transform have all-zero input and therefore zero output
    if (t < th) {
        int16_t* row = res + t * RS;
        switch (log2W) {
        case 2: row_pass<2>(row, w, rk, rect, rowShift, lossless); break;
        case 3: row_pass<3>(row, w, rk, rect, rowShift, lossless); break;
        case 4: row_pass<4>(row, w, rk, rect, rowShift, lossless); break;
        case 5: if constexpr (MAX >= 32) row_pass<5>(row, w, rk, rect, rowShift, lossless); break;
        default: if constexpr (MAX >= 64) row_pass<6>(row, w, rk, rect, rowShift, lossless); break;
        }
    } else if (t < h) {
        int16_t* row = res + t * RS;
        for (int j = 0; j < w; j++) row[j] = 0;
    }
    coop_sync<NT>();
    const int flipUD = type == AV1R_FLIPADST_DCT || type == AV1R_FLIPADST_ADST || type == AV1R_V_FLIPADST || type == AV1R_FLIPADST_FLIPADST;
    const int flipLR = type == AV1R_DCT_FLIPADST || type == AV1R_ADST_FLIPADST || type == AV1R_H_FLIPADST || type == AV1R_FLIPADST_FLIPADST;
    if (t < w) {
        const int16_t* col = res + t;
        int16_t* out = res + (flipLR ? w - 1 - t : t);
        switch (log2H) {
        case 2: col_pass<2, RS>(col, out, ck, colShift, lossless, flipUD); break;
        case 3: col_pass<3, RS>(col, out, ck, colShift, lossless, flipUD); break;
        case 4: col_pass<4, RS>(col, out, ck, colShift, lossless, flipUD); break;
        case 5: if constexpr (MAX >= 32) col_pass<5, RS>(col, out, ck, colShift, lossless, flipUD); break;
        default: if constexpr (MAX >= 64) col_pass<6, RS>(col, out, ck, colShift, lossless, flipUD); break;
        }
    }
    coop_sync<NT>();
}

// The prediction of an intra or palette transform block into L.pred (TransformBlock::decode,
// TransformBlock.cpp:2400-2420): palette colours (Block.cpp:2279-2298), or
// IntraPredict::predict_intra with CFL (IntraPredict.cpp:563-667).  Inter TBs predict
// nothing here (their prediction is already in the frame).  Ends with a coop_sync.
template <int NT, int MAX, bool COH>
DEV void tb_predict(const KParams& k, const WorkItem& tb, const DevBlock& blk, TbLds<MAX>& L, const GranEdges* G = nullptr,
    bool gran = false, int edgeFilter = -1)
{
    constexpr int CM = TbLds<MAX>::CM;
    const int t = coop_lane<NT>();
    const int plane = tb.plane, x = tb.x, y = tb.y, txSz = tb.tx_size;
    const int w = ctab<NT>(av1r_tx_w, txSz), h = ctab<NT>(av1r_tx_h, txSz);
    const int log2W = ctab<NT>(av1r_tx_w_log2, txSz), log2H = ctab<NT>(av1r_tx_h_log2, txSz);
    const DevPlane& dst = k.cur.pl[plane];
    const uint32_t bflags = blk.flags;
    if (tb.pred == AV1R_PRED_PALETTE) {
        const uint8_t* ph = k.palette + blk.palette_off;
        int bx = x - (blk.mi_col >> (plane ? 1 : 0)) * 4, by = y - (blk.mi_row >> (plane ? 1 : 0)) * 4;
        int mw = plane ? ph[2] : ph[0];
        const uint8_t* map = ph + AV1R_PALETTE_HDR + (plane ? ph[0] * ph[1] : 0);
        const uint8_t* colors = ph + 4 + 8 * plane;
        for (int q = t; q < w * h; q += NT) {
            int i = q >> log2W, j = q & (w - 1);
            L.pred[i * MAX + j] = colors[map[(by + i) * mw + bx + j]];
        }
    } else if (tb.pred == AV1R_PRED_INTRA) {
        if (COH && gran)
            coop_intra_edges_gran<NT>(k.mi_cols, k.mi_rows, dst, plane, x, y, log2W, log2H,
                (tb.flags & AV1R_TB_HAVE_LEFT) != 0, (tb.flags & AV1R_TB_HAVE_ABOVE) != 0,
                (tb.flags & AV1R_TB_HAVE_AR) != 0, (tb.flags & AV1R_TB_HAVE_BL) != 0, L.intra, *G);
        if (COH && gran) trace_stamp(G->tr, 8);
        if (!(COH && gran))
            coop_intra_edges<NT, COH>(k.mi_cols, k.mi_rows, dst, plane, x, y, log2W, log2H,
                (tb.flags & AV1R_TB_HAVE_LEFT) != 0, (tb.flags & AV1R_TB_HAVE_ABOVE) != 0,
                (tb.flags & AV1R_TB_HAVE_AR) != 0, (tb.flags & AV1R_TB_HAVE_BL) != 0, L.intra);
        const int isCfl = plane > 0 && blk.uv_mode == AV1R_UV_CFL_PRED;
        IntraParams P;
        P.plane = plane;
        P.x = x;
        P.y = y;
        P.log2W = log2W;
        P.log2H = log2H;
        P.haveLeft = (tb.flags & AV1R_TB_HAVE_LEFT) != 0;
        P.haveAbove = (tb.flags & AV1R_TB_HAVE_ABOVE) != 0;
        P.haveAR = (tb.flags & AV1R_TB_HAVE_AR) != 0;
        P.haveBL = (tb.flags & AV1R_TB_HAVE_BL) != 0;
        P.mode = plane == 0 ? blk.y_mode : (isCfl ? AV1R_DC_PRED : blk.uv_mode);
        P.angleDelta = plane == 0 ? blk.angle_delta_y : blk.angle_delta_uv;
        P.filterIntra = plane == 0 && (bflags & AV1R_BLK_FILTER_INTRA);
        P.filterIntraMode = blk.filter_intra_mode;
        P.smooth = plane ? ((bflags & (AV1R_BLK_SMOOTH_A_UV | AV1R_BLK_SMOOTH_L_UV)) != 0)
                         : ((bflags & (AV1R_BLK_SMOOTH_A_Y | AV1R_BLK_SMOOTH_L_Y)) != 0);
        P.edgeFilter = edgeFilter >= 0 ? edgeFilter : k.hdr->enable_intra_edge_filter;
        int s = 0;
        if (isCfl) {
            // predict_chroma_from_luma (IntraPredict.cpp:632-667): the luma loads go out
            // together with the edge loads
            const DevPlane& luma = k.cur.pl[0];
            const int maxLW = blk.max_luma_w, maxLH = blk.max_luma_h;
            // (flow read site: the same block's luma, written by earlier items of the launch:
            // sc1 loads after the done-flag wait in k_flow)
            for (int q = t; q < w * h; q += NT) {
                int i = q >> log2W, j = q & (w - 1);
                int ly = imin((y + i) << 1, maxLH - 2), lx = imin((x + j) << 1, maxLW - 2);
                const int v = (ldp<COH>(luma, lx, ly) + ldp<COH>(luma, lx + 1, ly) + ldp<COH>(luma, lx, ly + 1) +
                                  ldp<COH>(luma, lx + 1, ly + 1)) << 1;
                L.cfl[i * CM + j] = (int16_t)v;
                s += v;
            }
        }
        coop_sync<NT>();  // edges gathered
        coop_intra_from_edges<NT>(k.mi_cols, k.mi_rows, P, L.intra, L.pred, MAX, COH && gran ? G->tr : nullptr);
        if (isCfl) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
            if (NT > 64) {  // across the waves of the workgroup
                if (t == 0) L.sum = 0;
                coop_sync<NT>();
                if ((t & 63) == 0) atomicAdd(&L.sum, s);
                coop_sync<NT>();
                s = L.sum;
            }
            const int alpha = plane == 1 ? blk.cfl_alpha_u : blk.cfl_alpha_v;
            const int avg = r2(s, log2W + P.log2H);
            for (int q = t; q < w * h; q += NT) {
                int i = q >> log2W, j = q & (w - 1);
                int dc = L.pred[i * MAX + j];
                L.pred[i * MAX + j] = (uint8_t)clip1(dc + r2s(alpha * (L.cfl[i * CM + j] - avg), 6));
            }
        }
    }
    coop_sync<NT>();
}

// Add and clip (TransformBlock.cpp:2440-2456) four samples per lane with dword frame
// accesses: prediction from L.pred (intra / palette) or from the frame (inter), plus the
// residual in L.res when the TB has coefficients.
template <int NT, int MAX, bool COH>
DEV void tb_store(const KParams& k, const WorkItem& tb, TbLds<MAX>& L)
{
    constexpr int RS = TbLds<MAX>::RS;
    const int t = coop_lane<NT>();
    const int txSz = tb.tx_size;
    const int l2q = av1r_tx_w_log2[txSz] - 2;  // log2 of the dwords per row
    const int nq = (av1r_tx_w[txSz] * av1r_tx_h[txSz]) >> 2;
    const DevPlane& dst = k.cur.pl[tb.plane];
    const bool hasRes = tb.coef_cnt != 0;
    for (int q = t; q < nq; q += NT) {
        const int i = q >> l2q, j = (q & ((1 << l2q) - 1)) << 2;
        const uint32_t p = tb.pred == AV1R_PRED_INTER ? ldp4<COH>(dst, tb.x + j, tb.y + i)
                                                      : *reinterpret_cast<const uint32_t*>(&L.pred[i * MAX + j]);
        uint32_t o = p;
        if (hasRes) {
            const uint32_t r01 = *reinterpret_cast<const uint32_t*>(&L.res[i * RS + j]);
            const uint32_t r23 = *reinterpret_cast<const uint32_t*>(&L.res[i * RS + j + 2]);
            const int r[4] = {(int16_t)(r01 & 0xffff), (int16_t)(r01 >> 16), (int16_t)(r23 & 0xffff), (int16_t)(r23 >> 16)};
            o = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) o |= (uint32_t)clip1((int)((p >> (8 * b)) & 0xff) + r[b]) << (8 * b);
        }
        stp4<COH>(dst, tb.x + j, tb.y + i, o);
    }
}

// k_flow's add and store: as tb_store, with the residual quads (4 int16 each) of the TB's
// precomputed tile already in registers (loaded before the dependency wait)
template <int NT, int MAX>
struct ResQuads {
    static constexpr int N = (MAX * MAX / 4 + NT - 1) / NT;
    uint2 r[N];
};
// ro: the TB's residual tile offset (KParams::tb_res; ~0u: none), known to the caller
template <int NT, int MAX>
DEV void res_prefetch(const KParams& k, const WorkItem& tb, uint32_t ro, ResQuads<NT, MAX>& R)
{
    const int t = coop_lane<NT>();
    const int nq = (ctab<NT>(av1r_tx_w, tb.tx_size) * ctab<NT>(av1r_tx_h, tb.tx_size)) >> 2;
    const uint2* q4 = reinterpret_cast<const uint2*>(k.res + ro);
#pragma unroll
    for (int u = 0; u < ResQuads<NT, MAX>::N; u++) {
        const int q = t + u * NT;
        R.r[u] = (ro != ~0u && q < nq) ? q4[q] : make_uint2(0, 0);
    }
}
DEV uint32_t add4(uint32_t p, uint2 r)
{
    const int v[4] = {(int16_t)(r.x & 0xffff), (int16_t)(r.x >> 16), (int16_t)(r.y & 0xffff), (int16_t)(r.y >> 16)};
    uint32_t o = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) o |= (uint32_t)clip1((int)((p >> (8 * b)) & 0xff) + v[b]) << (8 * b);
    return o;
}
template <int NT, int MAX>
DEV void tb_store_flow(const KParams& k, const WorkItem& tb, TbLds<MAX>& L, const ResQuads<NT, MAX>& R, uint32_t epoch)
{
    const int t = coop_lane<NT>();
    const int l2q = ctab<NT>(av1r_tx_w_log2, tb.tx_size) - 2;
    const int tw = ctab<NT>(av1r_tx_w, tb.tx_size), th = ctab<NT>(av1r_tx_h, tb.tx_size);
    const int nq = (tw * th) >> 2;
    const DevPlane& dst = k.cur.pl[tb.plane];
    const bool gran = k.gran;
#pragma unroll
    for (int u = 0; u < ResQuads<NT, MAX>::N; u++) {
        const int q = t + u * NT;
        if (q < nq) {
            const int i = q >> l2q, j = (q & ((1 << l2q) - 1)) << 2;
            uint32_t* pp = reinterpret_cast<uint32_t*>(&L.pred[i * MAX + j]);
            const uint32_t o = add4(*pp, R.r[u]);
            stp4<true>(dst, tb.x + j, tb.y + i, o);
            if (gran) *pp = o;  // the final pixels, for the edge granules
        }
    }
    if (gran) {
        coop_sync<NT>();
        const int p = tb.plane;
        coop_publish_gran<NT>(L.pred, MAX, tb.x, tb.y, tw, th, k.gran_h[p], k.gran_v[p],
            k.gran_w[p], k.gran_hn[p], epoch);
    }
}

// One transform block of the level launches (TransformBlock::decode,
// TransformBlock.cpp:2400-2456): the prediction inputs are final before the launch.
template <int NT, int MAX>
DEV void tb_item(const KParams& k, const WorkItem& wi, TbLds<MAX>& L, unsigned long long* tr)
{
    const int t = coop_lane<NT>();
    const uint32_t c0 = t < wi.coef_cnt ? coef_at(k, wi.coef_off, wi.flags, t) : 0u;
    const DevBlock& blk = k.blocks[wi.block];
    tb_predict<NT, MAX, false>(k, wi, blk, L);
    trace_stamp(tr, 4);
    if (wi.coef_cnt) tb_residual<NT, MAX>(k, wi, blk, L.res, c0);
    trace_stamp(tr, 13);
    tb_store<NT, MAX, false>(k, wi, L);
}

// ---------------------------------------------------------------------------------
// Inter prediction
//
// Work item = one <= 32x32 luma tile (+ its 4:2:0 chroma) of an inter-coded block: every
// sample of Block::compute_prediction (decoder/Block.cpp:100-174) ->
// InterPredict::predict_inter (decoder/InterPredict.cpp:962-1049) depends only on its
// own position, so a 128x128 block becomes 16 independent tiles of identical cost.  Per
// tile and reference, the (h + 7) x (w + 7) reference window is staged in LDS with one
// sweep, the horizontal sub-pel pass runs once per window row into LDS, and the vertical
// pass produces each sample; warps stage their 15 x 8 intermediates per 8x8 block.  The
// compound blend is applied per sample and the tile is stored once.  Inter-intra blocks
// store their plain inter prediction here; ii_item blends the intra part once the
// block's edges are final.
// ---------------------------------------------------------------------------------
#define TS 32                     // tile edge (luma)
#define WC (TS + 8)               // window row stride
#define WARP_ROWS 16              // warped regions are predicted in chunks of 16 rows
#define HBN ((TS + 7) * TS)       // horizontal rows; >= warp intermediates (TS * WARP_ROWS / 64 * 120)

// LDS of one tile of edge TSZ: TS for k_inter, 8 for k_inter_s (four tiles per wave)
template <int TSZ>
struct InterLdsT {
    static constexpr int WCS = TSZ + 8;            // window row stride
    static constexpr int HBS = (TSZ + 7) * TSZ;    // >= warp intermediates (TSZ * min(TSZ, WARP_ROWS) / 64 * 120)
    uint8_t tile[TSZ * TSZ];      // this plane's tile, assembled before the store
    uint8_t mask[TSZ * TSZ];      // compute_prediction's Mask (luma, persists across planes)
    uint8_t win[2][(TSZ + 7) * WCS];  // reference windows (luma, or the current plane)
    struct {
        int16_t hbw[2][HBS];      // horizontally filtered window rows / warp intermediates
    } u;
};
using InterLds = InterLdsT<TS>;
static_assert(InterLdsT<TS>::HBS == HBN, "inter LDS");

// NT lanes per tile: 64 (k_inter: one tile per single-wave workgroup, workgroup barriers)
// or 16 (k_inter_s: four tiles per wave, wave-level ordering only -- the tiles of a wave
// take different paths, and a one-wave workgroup needs no s_barrier)
template <int NT>
DEV int il_lane() { return NT == 64 ? (int)threadIdx.x : (int)(threadIdx.x & (NT - 1)); }
template <int NT>
DEV void il_sync()
{
    if (NT == 64) __syncthreads();
    else coop_sync<NT>();
}

struct RefSel {
    DevPlane p;
    int lastX, lastY;
    int startX, startY, xStep, yStep;
    int filtX, filtY;  // subpel filter sets (getFilterIdx)
    int warp;          // 0 none, 1 local, 2 global
    int alpha, beta, gamma, delta;
    const int32_t* wp;
    int useWin;        // unscaled + not warped: LDS window path
    int scaled;        // FrameHeader::is_scaled (Parser.cpp:795-803)
};

// Block::LocalWarp::setupShear (Block.cpp:1179-1200) incl. resolveDivisor (:1087-1095)
DEV int setup_shear(const int32_t* wp, int& alpha, int& beta, int& gamma, int& delta)
{
    int alpha0 = CLIP3(-32768, 32767, wp[2] - (1 << 16));
    int beta0 = CLIP3(-32768, 32767, wp[3]);
    int64_t d = wp[2];
    int64_t ad = d < 0 ? -d : d;
    int n = floor_log2_u64((uint64_t)ad);
    int64_t e = ad - ((int64_t)1 << n);
    int64_t f = n > 8 ? r2_64(e, n - 8) : (e << (8 - n));
    int divShift = n + 14;
    int divFactor = d < 0 ? -(int)av1r_div_lut[f] : (int)av1r_div_lut[f];
    int64_t v = (int64_t)(wp[4] << 16);
    int gamma0 = CLIP3(-32768, 32767, (int)r2s_64(v * divFactor, divShift));
    int64_t w = (int64_t)(wp[3] * wp[4]);
    int delta0 = CLIP3(-32768, 32767, wp[5] - (int)r2s_64(w * divFactor, divShift) - (1 << 16));
    alpha = r2s(alpha0, 6) << 6;
    beta = r2s(beta0, 6) << 6;
    gamma = r2s(gamma0, 6) << 6;
    delta = r2s(delta0, 6) << 6;
    if ((4 * iabs(alpha) + 7 * iabs(beta)) >= (1 << 16)) return 0;
    if ((4 * iabs(gamma) + 4 * iabs(delta)) >= (1 << 16)) return 0;
    return 1;
}

DEV int filter_idx(int filt, int size, int dir)
{
    int f = dir ? (filt >> 4) : (filt & 15);
    if (size <= 4) {
        if (f == AV1R_EIGHTTAP || f == AV1R_EIGHTTAP_SHARP) return 4;
        if (f == AV1R_EIGHTTAP_SMOOTH) return 5;
    }
    return f;
}

// motionVectorScaling (InterPredict.cpp:66-83) + the ref geometry of blockInterPrediction
DEV void select_ref(const KParams& k, RefSel& R, int refIdx, int plane, int x, int y, const int16_t* mv)
{
    const int sub = plane ? 1 : 0;
    int rw, rh;
    if (refIdx < 0) {  // intra block copy predicts from the current (pre-filter) frame
        R.p = k.cur.pl[plane];
        rw = k.frame_w;
        rh = k.frame_h;
        R.lastX = ((k.mi_cols * 4 + sub) >> sub) - 1;
        R.lastY = ((k.mi_rows * 4 + sub) >> sub) - 1;
    } else {
        const DevFrame& f = k.ref[refIdx];
        R.p = f.pl[plane];
        rw = f.width;
        rh = f.height;
        R.lastX = ((rw + sub) >> sub) - 1;
        R.lastY = ((rh + sub) >> sub) - 1;
    }
    int xs = ((rw << 14) + (k.frame_w / 2)) / k.frame_w;
    int ys = ((rh << 14) + (k.frame_h / 2)) / k.frame_h;
    int origX = ((x << 4) + ((2 * mv[1]) >> sub) + 8);
    int origY = ((y << 4) + ((2 * mv[0]) >> sub) + 8);
    int baseX = origX * xs - (8 << 14);
    int baseY = origY * ys - (8 << 14);
    R.startX = r2s(baseX, 8) + 32;
    R.startY = r2s(baseY, 8) + 32;
    R.xStep = r2s(xs, 4);
    R.yStep = r2s(ys, 4);
    R.scaled = xs != (1 << 14) || ys != (1 << 14);
    R.warp = 0;
    R.useWin = 0;
}

// One predicted sample straight from the reference plane: blockPixelPredict /
// blockSubPixelPredict (InterPredict.cpp:319-383).  Used for scaled references.
DEV int pred_direct(const RefSel& R, int r, int c, int R0, int R1)
{
    if (!((R.startX >> 6) & 15) && !((R.startY >> 6) & 15)) {
        int xx = CLIP3(0, R.lastX, (R.startX >> 10) + c), yy = CLIP3(0, R.lastY, (R.startY >> 10) + r);
        return (int16_t)(R.p.p[(size_t)yy * R.p.stride + xx] << (14 - R0 - R1));
    }
    int p = R.startX + R.xStep * c;
    const int16_t* hf = av1r_subpel_filters + (R.filtX * 16 + ((p >> 6) & 15)) * 8;
    int x0 = (p >> 10) - 3;
    int pv = (R.startY & 1023) + R.yStep * r;
    const int16_t* vf = av1r_subpel_filters + (R.filtY * 16 + ((pv >> 6) & 15)) * 8;
    int ybase = (R.startY >> 10) + (pv >> 10) - 3;
    int s = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint8_t* row = R.p.p + (size_t)CLIP3(0, R.lastY, ybase + t) * R.p.stride;
        int hs = 0;
#pragma unroll
        for (int u = 0; u < 8; u++) hs += hf[u] * row[CLIP3(0, R.lastX, x0 + u)];
        s += vf[t] * r2(hs, R0);
    }
    return (int16_t)r2(s, R1);
}

// Stage the (rh + 7) x (rw + 7) reference window of PU-relative region
// [rx0, rx0 + rw) x [ry0, ry0 + rh) (3 left/above, 4 right/below filter margin), for rw,
// rh <= S.  Rows are clamped per row.  When no column needs clamping, each lane moves whole
// rows: one row is at most ND + 1 aligned source dwords, loaded at once (wide loads) and
// byte-aligned into ND window dwords -- a window costs one memory round trip (the earlier
// per-dword loop waited for each iteration's loads: two round trips per 8x8 luma window of
// k_inter_s, up to seven per 32x32 one of k_inter).  Otherwise byte by byte.  The last
// source dword of a row may lie up to 7 bytes past the window's right edge: inside the
// row's stride padding (planes carry a 64-pixel margin).
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
template <int NT = 64, int S = TS>
DEV void load_window(const RefSel& R, uint8_t* win, int rx0, int ry0, int rw, int rh, int wcs = WC)
{
    const int wx0 = (R.startX >> 10) - 3 + rx0, wy0 = (R.startY >> 10) - 3 + ry0;
    const int wc = rw + 7, wr = rh + 7;
    const int lane = il_lane<NT>();
    if (wx0 >= 0 && wx0 + wc - 1 <= R.lastX) {
        constexpr int ND = (S + 7 + 3) / 4;     // window dwords per row, at most
        constexpr int NV = (ND + 1 + 3) / 4;    // 16-byte source loads per row
        const int ndw = (wc + 3) >> 2;
        const uint32_t sh = (uint32_t)(wx0 & 3);
        const uint8_t* base = R.p.p + (wx0 & ~3);
        for (int i = lane; i < wr; i += NT) {
            const u32x4a4* src = reinterpret_cast<const u32x4a4*>(base + (size_t)CLIP3(0, R.lastY, wy0 + i) * R.p.stride);
            uint32_t v[4 * NV];
#pragma unroll
            for (int q = 0; q < NV; q++) {
                const u32x4a4 x = src[q];
                v[4 * q] = x.x;
                v[4 * q + 1] = x.y;
                v[4 * q + 2] = x.z;
                v[4 * q + 3] = x.w;
            }
            uint32_t* dst = reinterpret_cast<uint32_t*>(win + i * wcs);
#pragma unroll
            for (int d = 0; d < ND; d++)
                if (d < ndw) dst[d] = __builtin_amdgcn_alignbyte(v[d + 1], v[d], sh);
        }
        return;
    }
    for (int q = lane; q < wc * wr; q += NT) {
        int i = q / wc, j = q - i * wc;
        int yy = CLIP3(0, R.lastY, wy0 + i), xx = CLIP3(0, R.lastX, wx0 + j);
        win[i * wcs + j] = R.p.p[(size_t)yy * R.p.stride + xx];
    }
}

// The 8 taps of sub-pixel filter f (= set * 16 + phase, av1r_subpel_filters) packed for
// the dot-product passes.  Every AV1 sub-pixel tap is even (each filter sums to 128), so the
// horizontal pass takes them halved as signed bytes (taps 0-3 in .x, 4-7 in .y: every
// halved tap, 64 at phase 0 included, fits), and the vertical pass as int16 pairs.
DEV uint2 hfilt_pk(int f)
{
    const int16_t* c = av1r_subpel_filters + f * 8;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        lo |= (uint32_t)((c[u] >> 1) & 0xff) << (8 * u);
        hi |= (uint32_t)((c[u + 4] >> 1) & 0xff) << (8 * u);
    }
    return make_uint2(lo, hi);
}
DEV uint4 vfilt_pk(int f)
{
    const int16_t* c = av1r_subpel_filters + f * 8;
    auto pr = [&](int u) { return (uint32_t)(uint16_t)c[u] | ((uint32_t)(uint16_t)c[u + 1] << 16); };
    return make_uint4(pr(0), pr(2), pr(4), pr(6));
}
typedef short sp2 __attribute__((ext_vector_type(2)));
DEV int dot2_i16(uint32_t a, uint32_t b, int acc)
{
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(sp2, a), __builtin_bit_cast(sp2, b), acc, false);
}
DEV uint32_t vf_pair(const uint4& vf, int t) { return t == 0 ? vf.x : t == 1 ? vf.y : t == 2 ? vf.z : vf.w; }

// Horizontal pass of blockSubPixelPredict (InterPredict.cpp:340-362) over the (rh + 7)
// window rows: intermediate[r][c] = Round2(sum hf[t] * ref[r][c + t - 3], R0).  Four
// outputs per lane from three LDS dwords when rw is a multiple of 4, each two v_dot4 of the
// halved taps (hfilt_pk) with the pixels biased to signed bytes (p ^ 0x80 = p - 128):
// sum hf * p = 2 * sum (hf / 2) * (p - 128) + 128 * 128.
template <int NT = 64>
DEV void hpass(const uint8_t* win, int16_t* hb, int rw, int rh, uint2 hf, int R0, int wcs = WC, int hstr = TS)
{
    if ((rw & 3) == 0) {
        const int g4 = rw >> 2, lg = ilog2p(g4);  // (rw: a power of two)
        for (int q = il_lane<NT>(); q < (rh + 7) * g4; q += NT) {
            const int i = q >> lg, g = q & (g4 - 1);
            const uint32_t* w32 = reinterpret_cast<const uint32_t*>(win + i * wcs) + g;
            const uint32_t d0 = w32[0] ^ 0x80808080u, d1 = w32[1] ^ 0x80808080u, d2 = w32[2] ^ 0x80808080u;
            int o[4];
#pragma unroll
            for (int m = 0; m < 4; m++) {
                const uint32_t a = __builtin_amdgcn_alignbyte(d1, d0, (uint32_t)m);
                const uint32_t b = __builtin_amdgcn_alignbyte(d2, d1, (uint32_t)m);
                const int hs = 2 * __builtin_amdgcn_sdot4((int)b, (int)hf.y, __builtin_amdgcn_sdot4((int)a, (int)hf.x, 0, false), false) + 16384;
                o[m] = r2(hs, R0) & 0xffff;
            }
            uint2 v;
            v.x = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
            v.y = (uint32_t)o[2] | ((uint32_t)o[3] << 16);
            *reinterpret_cast<uint2*>(hb + i * hstr + 4 * g) = v;
        }
        return;
    }
    for (int q = il_lane<NT>(); q < (rh + 7) * rw; q += NT) {
        const int i = q / rw, j = q - i * rw;
        const uint8_t* row = win + i * wcs + j;
        int hs = 0;
#pragma unroll
        for (int u = 0; u < 8; u++) hs += 2 * (int)(int8_t)((u < 4 ? hf.x : hf.y) >> (8 * (u & 3))) * row[u];
        hb[i * hstr + j] = (int16_t)r2(hs, R0);
    }
}

// The same sample as pred_direct for an unscaled, unwarped reference: the vertical pass
// over the staged intermediate rows (or the integer-position copy from the window), the
// taps as int16 pairs (vfilt_pk) against row pairs: four v_dot2.
DEV int pred_win(const uint8_t* win, const int16_t* hb, int rr, int cc, int R0, int R1, const uint4& vf, int integer,
    int wcs = WC, int hstr = TS)
{
    if (integer) return (int16_t)(win[(rr + 3) * wcs + cc + 3] << (14 - R0 - R1));
    const int16_t* col = hb + rr * hstr + cc;
    int s = 0;
#pragma unroll
    for (int t = 0; t < 4; t++)
        s = dot2_i16((uint32_t)(uint16_t)col[2 * t * hstr] | ((uint32_t)(uint16_t)col[(2 * t + 1) * hstr] << 16), vf_pair(vf, t), s);
    return (int16_t)r2(s, R1);
}
// Four horizontally adjacent samples (cc a multiple of 4): 8 LDS reads of 4 int16, each
// column's row pairs gathered by v_perm into v_dot2 operands.
DEV void pred_win4(const uint8_t* win, const int16_t* hb, int rr, int cc, int R0, int R1, const uint4& vf, int integer, int* out,
    int wcs = WC, int hstr = TS)
{
    if (integer) {
#pragma unroll
        for (int m = 0; m < 4; m++) out[m] = (int16_t)(win[(rr + 3) * wcs + cc + 3 + m] << (14 - R0 - R1));
        return;
    }
    int s[4] = {0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const uint2 a = *reinterpret_cast<const uint2*>(hb + (rr + 2 * t) * hstr + cc);
        const uint2 b = *reinterpret_cast<const uint2*>(hb + (rr + 2 * t + 1) * hstr + cc);
        const uint32_t f = vf_pair(vf, t);
        s[0] = dot2_i16(__builtin_amdgcn_perm(b.x, a.x, 0x05040100u), f, s[0]);
        s[1] = dot2_i16(__builtin_amdgcn_perm(b.x, a.x, 0x07060302u), f, s[1]);
        s[2] = dot2_i16(__builtin_amdgcn_perm(b.y, a.y, 0x05040100u), f, s[2]);
        s[3] = dot2_i16(__builtin_amdgcn_perm(b.y, a.y, 0x07060302u), f, s[3]);
    }
#pragma unroll
    for (int m = 0; m < 4; m++) out[m] = (int16_t)r2(s[m], R1);
}

DEV void warp_origin(const RefSel& R, int i8, int j8, int puX, int puY, int sub, int& ix4, int& sx4, int& iy4, int& sy4)
{
    const int32_t* wp = R.wp;
    int srcX = (puX + j8 * 8 + 4) << sub;
    int srcY = (puY + i8 * 8 + 4) << sub;
    int dstX = wp[2] * srcX + wp[3] * srcY + wp[0];
    int dstY = wp[4] * srcX + wp[5] * srcY + wp[1];
    int x4 = dstX >> sub, y4 = dstY >> sub;
    ix4 = x4 >> 16;
    sx4 = x4 & 0xffff;
    iy4 = y4 >> 16;
    sy4 = y4 & 0xffff;
}
template <int NT = 64>
DEV void warp_hpass(const RefSel& R, int16_t* hb, int rx0, int ry0, int rw, int rh, int puX, int puY, int sub, int R0)
{
    const int w8 = rw >> 3, nb = (rh >> 3) * w8;
    for (int q = il_lane<NT>(); q < nb * 120; q += NT) {
        const int b = q / 120, e = q - b * 120;
        const int bi = b / w8;
        const int i8 = (ry0 >> 3) + bi, j8 = (rx0 >> 3) + (b - bi * w8);
        int ix4, sx4, iy4, sy4;
        warp_origin(R, i8, j8, puX, puY, sub, ix4, sx4, iy4, sy4);
        const int i1 = (e >> 3) - 7, i2 = (e & 7) - 4;
        const int sx = sx4 + R.alpha * i2 + R.beta * i1;
        const int8_t* hf = av1r_warped_filters + (r2(sx, 10) + 64) * 8;
        const uint8_t* row = R.p.p + (size_t)CLIP3(0, R.lastY, iy4 + i1) * R.p.stride;
        int hs = 0;
#pragma unroll
        for (int k3 = 0; k3 < 8; k3++) hs += hf[k3] * row[CLIP3(0, R.lastX, ix4 + i2 - 3 + k3)];
        hb[q] = (int16_t)r2(hs, R0);
    }
}
DEV int warp_v(const RefSel& R, const int16_t* hb, int rr, int cc, int r, int c, int rw, int puX, int puY, int sub, int R1)
{
    int ix4, sx4, iy4, sy4;
    warp_origin(R, r >> 3, c >> 3, puX, puY, sub, ix4, sx4, iy4, sy4);
    const int i1 = (r & 7) - 4, i2 = (c & 7) - 4;
    const int sy = sy4 + R.gamma * i2 + R.delta * i1;
    const int8_t* vf = av1r_warped_filters + (r2(sy, 10) + 64) * 8;
    const int16_t* col = hb + ((rr >> 3) * (rw >> 3) + (cc >> 3)) * 120 + (r & 7) * 8 + (c & 7);
    int s = 0;
#pragma unroll
    for (int i3 = 0; i3 < 8; i3++) s += vf[i3] * col[i3 * 8];
    return (int16_t)r2(s, R1);
}

DEV int wedge_oblique63(int i, int j)
{
    int shift = 16 - (i >> 1);
    return (i & 1) ? av1r_wedge_master_oblique_odd[CLIP3(0, 63, j - (shift - 1))]
                   : av1r_wedge_master_oblique_even[CLIP3(0, 63, j - shift)];
}
DEV int wedge_master(int dir, int i, int j)
{
    // MasterMask (InterPredict.cpp:835-858) evaluated on the fly
    switch (dir) {
    case AV1R_WEDGE_VERTICAL: return av1r_wedge_master_vertical[j];
    case AV1R_WEDGE_HORIZONTAL: return av1r_wedge_master_vertical[i];
    case AV1R_WEDGE_OBLIQUE63: return wedge_oblique63(i, j);
    case AV1R_WEDGE_OBLIQUE27: return wedge_oblique63(j, i);
    case AV1R_WEDGE_OBLIQUE117: return 64 - wedge_oblique63(i, 63 - j);
    default: return 64 - wedge_oblique63(j, 63 - i);  // OBLIQUE153
    }
}

struct WedgeSel {
    int dir, xoff, yoff, flip;
};
template <int NT = 64>
DEV WedgeSel wedge_select(int bs, int wedge)
{
    int w = av1r_num4x4w[bs] * 4, h = av1r_num4x4h[bs] * 4;
    int shape = h > w ? 0 : (h < w ? 1 : 2);
    const uint8_t* cb = av1r_wedge_codebook[shape][wedge];
    WedgeSel s;
    s.dir = cb[0];
    s.xoff = 32 - ((cb[1] * w) >> 3);
    s.yoff = 32 - ((cb[2] * h) >> 3);
    // flipSign (initialise_wedge_mask_table, InterPredict.cpp:870-877)
    // (the w + h - 1 edge samples summed across the tile's NT lanes; call with all of them active)
    int sum = 0;
    for (int i = threadIdx.x & (NT - 1); i < w + h - 1; i += NT)
        sum += i < w ? wedge_master(s.dir, s.yoff, s.xoff + i) : wedge_master(s.dir, s.yoff + i - w + 1, s.xoff);
#pragma unroll
    for (int o = NT / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o, NT);
    int avg = (sum + (w + h - 1) / 2) / (w + h - 1);
    s.flip = avg < 32;
    return s;
}

// getDistanceWeights (InterPredict.cpp:917-960)
// The mode info a prediction unit of block `blk` uses: the block's own, which its record
// carries (loaded with the record: no dependent load), unless a sub-8x8 chroma unit takes a
// neighbour's from the mode-info grid (Block.cpp:146-174)
struct PuInfo {
    int16_t mv[2][2];
    int8_t ref_frame[2];
    uint8_t filt;
};
DEV PuInfo pu_info(const KParams& k, const DevBlock& blk, int candRow, int candCol)
{
    PuInfo p;
    if (candRow == blk.mi_row && candCol == blk.mi_col) {
#pragma unroll
        for (int l = 0; l < 2; l++) {
            p.mv[l][0] = blk.mv[l][0];
            p.mv[l][1] = blk.mv[l][1];
            p.ref_frame[l] = blk.ref_frame[l];
        }
        p.filt = blk.filt;
    } else {
        const av1r_mi& m = mi_at(k, candRow, candCol);
#pragma unroll
        for (int l = 0; l < 2; l++) {
            p.mv[l][0] = m.mv[l][0];
            p.mv[l][1] = m.mv[l][1];
            p.ref_frame[l] = m.ref_frame[l];
        }
        p.filt = m.filt;
    }
    return p;
}

template <class MI>
DEV void distance_weights(const KParams& k, const MI& info, int& fwd, int& bck)
{
    int d1 = k.hdr->ref_dist[info.ref_frame[0] & 7];
    int d0 = k.hdr->ref_dist[info.ref_frame[1] & 7];
    int order = d0 <= d1;
    if (d0 == 0 || d1 == 0) {
        fwd = av1r_quant_dist_lookup[3][order];
        bck = av1r_quant_dist_lookup[3][1 - order];
        return;
    }
    int i;
    for (i = 0; i < 3; i++) {
        int c0 = av1r_quant_dist_weight[i][order], c1 = av1r_quant_dist_weight[i][1 - order];
        if (order) {
            if (d0 * c0 > d1 * c1) break;
        } else {
            if (d0 * c0 < d1 * c1) break;
        }
    }
    fwd = av1r_quant_dist_lookup[i][order];
    bck = av1r_quant_dist_lookup[i][1 - order];
}

// predict_inter for the PU-relative region [rx0, rx0 + rw) x [ry0, ry0 + rh) of the
// w x h prediction unit at plane position (x, y); sample (r, c) of the PU lands in
// L.tile[(toy + r) * TS + tox + c].  Ends with a barrier.
// The references of one prediction unit (predict_inter, InterPredict.cpp:962-1021):
// motion vector scaling, warp choice (local / global, Block.cpp:1179-1200) and filters.
// Returns isCompound.
DEV int setup_refs(const KParams& k, const DevBlock& blk, int plane, int x, int y, int w, int h,
    int candRow, int candCol, RefSel* R, const int32_t* lw)
{
    const av1r_frame_hdr& hd = *k.hdr;
    const PuInfo info = pu_info(k, blk, candRow, candCol);
    const int isCompound = info.ref_frame[1] > AV1R_INTRA_FRAME;
    const int isIntrabc = (blk.flags & AV1R_BLK_INTRABC) != 0;
    const int isGlobalMode = blk.y_mode == AV1R_GLOBALMV || blk.y_mode == AV1R_GLOBAL_GLOBALMV;
    int globalValid = 0;
#pragma unroll
    for (int l = 0; l < 2; l++) {
        if (l > isCompound) break;
        int refFrame = info.ref_frame[l];
        int a, b, c, d;
        if (isGlobalMode && hd.gm_type[refFrame & 7] > AV1R_GM_TRANSLATION)
            globalValid = setup_shear(hd.gm_params[refFrame & 7], a, b, c, d);
        int refIdx = isIntrabc ? -1 : hd.ref_frame_idx[refFrame - 1];
        select_ref(k, R[l], refIdx, plane, x, y, info.mv[l]);
        if (!(w < 8 || h < 8) && !hd.force_integer_mv) {
            if (blk.motion_mode == AV1R_LOCALWARP && (blk.flags & AV1R_BLK_LOCAL_VALID)) {
                R[l].warp = 1;
                R[l].wp = lw;  // (the block record in memory: blk may be a register copy)
            } else if (isGlobalMode && hd.gm_type[refFrame & 7] > AV1R_GM_TRANSLATION && globalValid
                && !R[l].scaled) {
                R[l].warp = 2;
                R[l].wp = hd.gm_params[refFrame & 7];
            }
        }
        if (R[l].warp) setup_shear(R[l].wp, R[l].alpha, R[l].beta, R[l].gamma, R[l].delta);
        R[l].filtX = filter_idx(info.filt, w, 1);
        R[l].filtY = filter_idx(info.filt, h, 0);
        R[l].useWin = !R[l].warp && R[l].xStep == 1024 && R[l].yStep == 1024;
    }
    return isCompound;
}

// predict_inter for the PU-relative region [rx0, rx0 + rw) x [ry0, ry0 + rh) of the
// w x h prediction unit at plane position (x, y); sample (r, c) of the PU lands in
// L.tile[(toy + r) * TS + tox + c].  Ends with a barrier.
template <int NT, int TSZ>
DEV void predict_pu(const KParams& k, const DevBlock& blk, InterLdsT<TSZ>& L, int plane, int x, int y,
    int w, int h, int candRow, int candCol, int rx0, int ry0, int rw, int rh, int tox, int toy, const int32_t* lw)
{
    const int t = il_lane<NT>();
    const PuInfo info = pu_info(k, blk, candRow, candCol);
    const int sub = plane ? 1 : 0;
    RefSel R[2];
    const int isCompound = setup_refs(k, blk, plane, x, y, w, h, candRow, candCol, R, lw);
    const int R0 = 3, R1 = isCompound ? 7 : 11, PostRound = 14 - (R0 + R1);
    uint2 hf[2];
    uint4 vf[2];
    int integer[2];
#pragma unroll
    for (int l = 0; l < 2; l++) {
        if (l > isCompound) break;
        const int hph = (R[l].startX >> 6) & 15, vph = (R[l].startY >> 6) & 15;
        integer[l] = !hph && !vph;
        hf[l] = hfilt_pk(R[l].filtX * 16 + hph);
        vf[l] = vfilt_pk(R[l].filtY * 16 + vph);
    }
    const int ct = blk.compound_type;
    int mode;  // 0 single reference (inter-intra: blended later by ii_item), 1 average, 2 distance, 3 mask
    if (!isCompound) mode = 0;
    else if (ct == AV1R_COMPOUND_AVERAGE) mode = 1;
    else if (ct == AV1R_COMPOUND_DISTANCE) mode = 2;
    else mode = 3;
    int fwd = 0, bck = 0;
    if (mode == 2) distance_weights(k, info, fwd, bck);
    WedgeSel ws = {0, 0, 0, 0};
    if (mode == 3 && ct == AV1R_COMPOUND_WEDGE) ws = wedge_select<NT>(blk.mi_size, blk.wedge_index);
    const int diffwtdLuma = ct == AV1R_COMPOUND_DIFFWTD && plane == 0;

    // a warped region goes in chunks of WARP_ROWS rows (its 15 x 8 intermediates per 8x8
    // block would not fit the LDS budget of 16 workgroups per CU otherwise)
    const int chunkH = (R[0].warp || (isCompound && R[1].warp)) ? WARP_ROWS : rh;
    const int ryA = ry0, rhA = rh;
    for (int cy = 0; cy < rhA; cy += chunkH) {
    const int ry0 = ryA + cy, rh = imin(chunkH, rhA - cy);  // this chunk
    if (R[0].useWin) load_window<NT, TSZ>(R[0], L.win[0], rx0, ry0, rw, rh, L.WCS);
    if (isCompound && R[1].useWin) load_window<NT, TSZ>(R[1], L.win[1], rx0, ry0, rw, rh, L.WCS);
    il_sync<NT>();
    if (R[0].useWin && !integer[0]) hpass<NT>(L.win[0], L.u.hbw[0], rw, rh, hf[0], R0, L.WCS, TSZ);
    if (R[0].warp) warp_hpass<NT>(R[0], L.u.hbw[0], rx0, ry0, rw, rh, x, y, sub, R0);
    if (isCompound && R[1].useWin && !integer[1]) hpass<NT>(L.win[1], L.u.hbw[1], rw, rh, hf[1], R0, L.WCS, TSZ);
    if (isCompound && R[1].warp) warp_hpass<NT>(R[1], L.u.hbw[1], rx0, ry0, rw, rh, x, y, sub, R0);
    il_sync<NT>();
    auto blend = [&](int p0, int p1, int r, int c) {
        int v;
        if (mode == 0) {
            v = clip1(p0);
        } else if (mode == 1) {
            v = clip1(r2(p0 + p1, 1 + PostRound));
        } else if (mode == 2) {
            v = clip1(r2(fwd * p0 + bck * p1, 4 + PostRound));
        } else {
            // mask (wedgeMask / differenceWeightMask) and maskBlend (InterPredict.cpp:555-609);
            // mask blocks are single-PU, so PU and block coordinates coincide
            int m;
            if (diffwtdLuma) {
                int diff = (int16_t)iabs(p0 - p1);
                diff = r2(diff, PostRound);
                int mm = CLIP3(0, 64, 38 + diff / 16);
                m = blk.mask_type ? 64 - mm : mm;
                L.mask[(toy + r) * TSZ + tox + c] = (uint8_t)m;
            } else if (!sub) {
                if (ct == AV1R_COMPOUND_WEDGE) {
                    int mv = wedge_master(ws.dir, ws.yoff + r, ws.xoff + c);
                    m = blk.wedge_sign == ws.flip ? mv : 64 - mv;
                } else {
                    m = L.mask[(toy + r) * TSZ + tox + c];
                }
            } else {
                // 4:2:0 chroma: average of the 2x2 luma-resolution mask entries
                int s4 = 0;
#pragma unroll
                for (int dy = 0; dy < 2; dy++)
#pragma unroll
                    for (int dx = 0; dx < 2; dx++) {
                        int mv;
                        if (ct == AV1R_COMPOUND_WEDGE) {
                            int mw = wedge_master(ws.dir, ws.yoff + 2 * r + dy, ws.xoff + 2 * c + dx);
                            mv = blk.wedge_sign == ws.flip ? mw : 64 - mw;
                        } else {
                            mv = L.mask[(2 * (toy + r) + dy) * TSZ + 2 * (tox + c) + dx];
                        }
                        s4 += mv;
                    }
                m = r2(s4, 2);
            }
            v = clip1(r2(m * p0 + (64 - m) * p1, 6 + PostRound));
        }
        L.tile[(toy + r) * TSZ + tox + c] = (uint8_t)v;
    };
    auto sample = [&](int l, int rr, int cc) {
        const int r = ry0 + rr, c = rx0 + cc;
        return R[l].useWin ? pred_win(L.win[l], L.u.hbw[l], rr, cc, R0, R1, vf[l], integer[l], L.WCS, TSZ)
             : R[l].warp   ? warp_v(R[l], L.u.hbw[l], rr, cc, r, c, rw, x, y, sub, R1)
                           : pred_direct(R[l], r, c, R0, R1);
    };
    if ((rw & 3) == 0 && R[0].useWin && (!isCompound || R[1].useWin)) {
        // four adjacent samples per lane (window references only)
        const int g4 = rw >> 2, lg = ilog2p(g4);  // (rw: a power of two)
        for (int q = t; q < rh * g4; q += NT) {
            const int rr = q >> lg, cc = (q & (g4 - 1)) * 4;
            int p0[4], p1[4] = {0, 0, 0, 0};
            pred_win4(L.win[0], L.u.hbw[0], rr, cc, R0, R1, vf[0], integer[0], p0, L.WCS, TSZ);
            if (isCompound) pred_win4(L.win[1], L.u.hbw[1], rr, cc, R0, R1, vf[1], integer[1], p1, L.WCS, TSZ);
            // one blend body, the four samples rotated through it (no unrolled copies)
            int a0 = p0[0], a1 = p0[1], a2 = p0[2], a3 = p0[3];
            int b0 = p1[0], b1 = p1[1], b2 = p1[2], b3 = p1[3];
#pragma nounroll
            for (int m = 0; m < 4; m++) {
                blend(a0, b0, ry0 + rr, rx0 + cc + m);
                a0 = a1; a1 = a2; a2 = a3;
                b0 = b1; b1 = b2; b2 = b3;
            }
        }
    } else {
        const int lw = ilog2p(rw);
        for (int q = t; q < rw * rh; q += NT) {
            const int rr = q >> lw, cc = q & (rw - 1);
            blend(sample(0, rr, cc), isCompound ? sample(1, rr, cc) : 0, ry0 + rr, rx0 + cc);
        }
    }
    il_sync<NT>();
    }
}

// Both chroma planes of a single-PU, unwarped, unscaled block at once (the common case of
// predict_pu for planes 1 and 2): the four reference windows (U, V x both references)
// are fetched in one round trip and each pass runs for both planes between the same two
// barriers, instead of one window round trip and three barriers per plane.  The tile
// region is [rx0, rx0 + rw) x [ry0, ry0 + rh) of the block (rw a multiple of 4); plane p
// lands in L.tile + p * C2_TILE.  Returns false, before touching LDS, when a reference is
// warped or scaled (the caller then predicts plane by plane).
#define C2_WS 24                   // chroma window row stride (<= 16 + 7 columns)
#define C2_WIN (23 * C2_WS)        // one chroma window (<= 16 + 7 rows)
#define C2_HS 16                   // chroma intermediate row stride
#define C2_HB (23 * C2_HS)         // one chroma intermediate
#define C2_TILE (16 * TS)          // chroma tile of plane 2 after plane 1's
DEV bool predict_chroma2(const KParams& k, const DevBlock& blk, InterLds& L, int x, int y, int w, int h, int rx0,
    int ry0, int rw, int rh, const int32_t* lw)
{
    const int t = threadIdx.x;
    const PuInfo info = pu_info(k, blk, blk.mi_row, blk.mi_col);
    RefSel R[2][2];
    const int isCompound = setup_refs(k, blk, 1, x, y, w, h, blk.mi_row, blk.mi_col, R[0], lw);
    if (!R[0][0].useWin || (isCompound && !R[0][1].useWin)) return false;
    setup_refs(k, blk, 2, x, y, w, h, blk.mi_row, blk.mi_col, R[1], lw);
    const int R0 = 3, R1 = isCompound ? 7 : 11, PostRound = 14 - (R0 + R1);
    uint2 hf[2];
    uint4 vf[2];
    int integer[2] = {1, 1};
#pragma unroll
    for (int l = 0; l < 2; l++) {
        if (l > isCompound) break;
        const int hph = (R[0][l].startX >> 6) & 15, vph = (R[0][l].startY >> 6) & 15;
        integer[l] = !hph && !vph;
        hf[l] = hfilt_pk(R[0][l].filtX * 16 + hph);
        vf[l] = vfilt_pk(R[0][l].filtY * 16 + vph);
    }
    const int ct = blk.compound_type;
    int mode;  // as predict_pu
    if (!isCompound) mode = 0;
    else if (ct == AV1R_COMPOUND_AVERAGE) mode = 1;
    else if (ct == AV1R_COMPOUND_DISTANCE) mode = 2;
    else mode = 3;
    int fwd = 0, bck = 0;
    if (mode == 2) distance_weights(k, info, fwd, bck);
    WedgeSel ws = {0, 0, 0, 0};
    if (mode == 3 && ct == AV1R_COMPOUND_WEDGE) ws = wedge_select(blk.mi_size, blk.wedge_index);
    uint8_t* win = &L.win[0][0];
    int16_t* hb = &L.u.hbw[0][0];
#pragma unroll
    for (int p = 0; p < 2; p++)
#pragma unroll
        for (int l = 0; l < 2; l++)
            if (l <= isCompound) load_window<64, 16>(R[p][l], win + (p * 2 + l) * C2_WIN, rx0, ry0, rw, rh, C2_WS);
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 2; p++)
#pragma unroll
        for (int l = 0; l < 2; l++)
            if (l <= isCompound && !integer[l])
                hpass(win + (p * 2 + l) * C2_WIN, hb + (p * 2 + l) * C2_HB, rw, rh, hf[l], R0, C2_WS, C2_HS);
    __syncthreads();
    const int g4 = rw >> 2;
    for (int q = t; q < 2 * rh * g4; q += 64) {
        const int p = q >= rh * g4, e = q - p * rh * g4;
        const int rr = e / g4, cc = (e - rr * g4) * 4;
        int p0[4], p1[4] = {0, 0, 0, 0};
        pred_win4(win + (p * 2) * C2_WIN, hb + (p * 2) * C2_HB, rr, cc, R0, R1, vf[0], integer[0], p0, C2_WS, C2_HS);
        if (isCompound)
            pred_win4(win + (p * 2 + 1) * C2_WIN, hb + (p * 2 + 1) * C2_HB, rr, cc, R0, R1, vf[1], integer[1], p1, C2_WS, C2_HS);
        uint8_t* tile = L.tile + p * C2_TILE;
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const int r = ry0 + rr, c = rx0 + cc + m;  // block-relative
            int v;
            if (mode == 0) {
                v = clip1(p0[m]);
            } else if (mode == 1) {
                v = clip1(r2(p0[m] + p1[m], 1 + PostRound));
            } else if (mode == 2) {
                v = clip1(r2(fwd * p0[m] + bck * p1[m], 4 + PostRound));
            } else {
                // 4:2:0 chroma mask: average of the 2x2 luma-resolution entries (maskBlend,
                // InterPredict.cpp:584-609); the luma pass left the diff-weighted mask in L.mask
                int s4 = 0;
#pragma unroll
                for (int dy = 0; dy < 2; dy++)
#pragma unroll
                    for (int dx = 0; dx < 2; dx++) {
                        int mv;
                        if (ct == AV1R_COMPOUND_WEDGE) {
                            int mw = wedge_master(ws.dir, ws.yoff + 2 * r + dy, ws.xoff + 2 * c + dx);
                            mv = blk.wedge_sign == ws.flip ? mw : 64 - mw;
                        } else {
                            mv = L.mask[(2 * rr + dy) * TS + 2 * (cc + m) + dx];
                        }
                        s4 += mv;
                    }
                const int mk = r2(s4, 2);
                v = clip1(r2(mk * p0[m] + (64 - mk) * p1[m], 6 + PostRound));
            }
            tile[rr * TS + cc + m] = (uint8_t)v;
        }
    }
    __syncthreads();
    return true;
}

// overlappedMotionCompensation (InterPredict.cpp:611-709) restricted to the tile
// [TX0, TX0 + TW) x [TY0, TY0 + TH) (block-relative plane coordinates).
template <int NT, int TSZ>
DEV void obmc(const KParams& k, const DevBlock& blk, InterLdsT<TSZ>& L, int plane, int baseX, int baseY, int w, int h,
    int TX0, int TY0, int TW, int TH)
{
    const int t = il_lane<NT>();
    const int sub = plane ? 1 : 0;
    const int bs = blk.mi_size;
    const av1r_frame_hdr& hd = *k.hdr;
    for (int pass = 0; pass < 2; pass++) {
        if (pass == 0 && !((blk.flags & AV1R_BLK_AVAIL_U) && plane_bsize(bs, plane) >= AV1R_BLOCK_8X8)) continue;
        if (pass == 1 && !(blk.flags & AV1R_BLK_AVAIL_L)) continue;
        const int n4 = pass ? av1r_num4x4h[bs] : av1r_num4x4w[bs];
        const int nLimit = imin(4, pass ? av1r_mih_log2[bs] : av1r_miw_log2[bs]);
        const int lim = pass ? imin(k.mi_rows, blk.mi_row + n4) : imin(k.mi_cols, blk.mi_col + n4);
        int pos4 = pass ? blk.mi_row : blk.mi_col;
        int nCount = 0;
        while (nCount < nLimit && pos4 < lim) {
            int candRow = pass ? (pos4 | 1) : blk.mi_row - 1;
            int candCol = pass ? blk.mi_col - 1 : (pos4 | 1);
            const av1r_mi& info = mi_at(k, candRow, candCol);
            int step4 = CLIP3(2, 16, pass ? av1r_num4x4h[info.mi_size] : av1r_num4x4w[info.mi_size]);
            if (info.ref_frame[0] > AV1R_INTRA_FRAME) {
                nCount++;
                int x4 = pass ? blk.mi_col : pos4, y4 = pass ? pos4 : blk.mi_row;
                int predW = pass ? imin(w >> 1, 32 >> sub) : imin(w, (step4 * 4) >> sub);
                int predH = pass ? imin(h, (step4 * 4) >> sub) : imin(h >> 1, 32 >> sub);
                int len = pass ? predW : predH;
                const uint8_t* mask = av1r_obmc_mask + (len == 2 ? 0 : len == 4 ? 2 : len == 8 ? 6 : len == 16 ? 14 : 30);
                int predX = (x4 * 4) >> sub, predY = (y4 * 4) >> sub;
                const int ox = predX - baseX, oy = predY - baseY;
                const int ix0 = imax(ox, TX0), ix1 = imin(ox + predW, TX0 + TW);
                const int iy0 = imax(oy, TY0), iy1 = imin(oy + predH, TY0 + TH);
                if (ix0 < ix1 && iy0 < iy1) {
                    const int rx0 = ix0 - ox, ry0 = iy0 - oy, rw = ix1 - ix0, rh = iy1 - iy0;
                    RefSel R;
                    select_ref(k, R, hd.ref_frame_idx[info.ref_frame[0] - 1], plane, predX, predY, info.mv[0]);
                    R.filtX = filter_idx(info.filt, predW, 1);
                    R.filtY = filter_idx(info.filt, predH, 0);
                    R.useWin = R.xStep == 1024 && R.yStep == 1024;
                    const int hph = (R.startX >> 6) & 15, vph = (R.startY >> 6) & 15;
                    const int integer = !hph && !vph;
                    const uint2 hf = hfilt_pk(R.filtX * 16 + hph);
                    const uint4 vf = vfilt_pk(R.filtY * 16 + vph);
                    if (R.useWin) {
                        load_window<NT, TSZ>(R, L.win[0], rx0, ry0, rw, rh, L.WCS);
                        il_sync<NT>();
                        if (!integer) hpass<NT>(L.win[0], L.u.hbw[0], rw, rh, hf, 3, L.WCS, TSZ);
                        il_sync<NT>();
                    }
                    const int lw = ilog2p(rw);
                    for (int q = t; q < rw * rh; q += NT) {
                        const int rr = q >> lw, cc = q & (rw - 1), i = ry0 + rr, j = rx0 + cc;
                        int p = R.useWin ? pred_win(L.win[0], L.u.hbw[0], rr, cc, 3, 11, vf, integer, L.WCS, TSZ)
                                         : pred_direct(R, i, j, 3, 11);
                        int m = pass ? mask[j] : mask[i];
                        uint8_t& d = L.tile[(oy + i - TY0) * TSZ + ox + j - TX0];
                        d = (uint8_t)clip1(r2(m * d + (64 - m) * clip1(p), 6));
                    }
                    il_sync<NT>();
                }
            }
            pos4 += step4;
        }
    }
}

// One tile (tx, ty) of inter block `bi`: all planes.
struct PlaneGeo {
    int baseX, baseY, pw, ph;      // the block in this plane
    int TX0, TY0, TW, TH;          // the tile, block-relative
    int candRow, candCol, predW, predH;  // prediction units (Block.cpp:146-174)
};
template <int TSZ>
DEV PlaneGeo plane_geo(const KParams& k, const DevBlock& blk, int plane, int tx, int ty)
{
    PlaneGeo G;
    const int bs = blk.mi_size;
    const int psz = plane_bsize(bs, plane);
    const int n4w = av1r_num4x4w[psz], n4h = av1r_num4x4h[psz];
    const int sub = plane ? 1 : 0;
    G.baseX = (blk.mi_col >> sub) * 4;
    G.baseY = (blk.mi_row >> sub) * 4;
    G.pw = n4w * 4;
    G.ph = n4h * 4;
    G.TX0 = (tx * TSZ) >> sub;
    G.TY0 = (ty * TSZ) >> sub;
    G.TW = imin(TSZ >> sub, G.pw - G.TX0);
    G.TH = imin(TSZ >> sub, G.ph - G.TY0);
    // sub-8x8 chroma may gather several prediction units
    G.candRow = (blk.mi_row >> sub) << sub;
    G.candCol = (blk.mi_col >> sub) << sub;
    G.predW = (av1r_num4x4w[bs] * 4) >> sub;
    G.predH = (av1r_num4x4h[bs] * 4) >> sub;
    int someUseIntra = 0;
    // only a sub-8x8 chroma block can change its PU layout (otherwise the gathered
    // geometry equals the block's own)
    if (G.predW != G.pw || G.predH != G.ph || G.candRow != blk.mi_row || G.candCol != blk.mi_col)
        for (int r = 0; r < (n4h << sub); r++)
            for (int c = 0; c < (n4w << sub); c++)
                if (mi_at(k, G.candRow + r, G.candCol + c).ref_frame[0] == AV1R_INTRA_FRAME) someUseIntra = 1;
    if (someUseIntra) {
        G.predW = G.pw;
        G.predH = G.ph;
        G.candRow = blk.mi_row;
        G.candCol = blk.mi_col;
    }
    return G;
}

// One tile (tx, ty) of inter block `bi`: all planes.
template <int NT, int TSZ>
DEV void inter_tile(const KParams& k, uint32_t bi, int tx, int ty, InterLdsT<TSZ>& L, unsigned long long* tr)
{
    const int t = il_lane<NT>();
    // the block record in scalar registers (one scalar load: a tile's fields are uniform)
    const DevBlock blk = sload(k.blocks + bi);
    const int32_t* lw = (blk.flags & AV1R_BLK_LOCAL_VALID) ? k.bext + 8 * (size_t)blk.palette_off : nullptr;
    const int nPl = (blk.flags & AV1R_BLK_HAS_CHROMA) ? 3 : 1;
    // timeline (-DAV1R_TRACE): 1 = block size | motion mode << 8 | compound << 12, 8 + plane
    // after each plane's store, 11 after the luma geometry, 12 after the luma prediction
    trace_put(tr, 1, blk.mi_size | (blk.motion_mode << 8) |
        ((mi_at(k, blk.mi_row, blk.mi_col).ref_frame[1] > AV1R_INTRA_FRAME) << 12));
    for (int plane = 0; plane < nPl; plane++) {
        const PlaneGeo G = plane_geo<TSZ>(k, blk, plane, tx, ty);
        if (plane == 0) trace_stamp(tr, 11);
        if constexpr (TSZ == TS) {
            if (plane == 1 && G.predW == G.pw && G.predH == G.ph && G.candRow == blk.mi_row && G.candCol == blk.mi_col &&
                blk.motion_mode != AV1R_OBMC_CAUSAL && !(G.TW & 3) &&
                predict_chroma2(k, blk, L, G.baseX, G.baseY, G.pw, G.ph, G.TX0, G.TY0, G.TW, G.TH, lw)) {
                // (G.TW a multiple of 4: a dword per lane and row quad; x, TX0 multiples of 4)
                const int lq = ilog2p(G.TW >> 2), nq = (G.TW * G.TH) >> 2;
                for (int q = t; q < 2 * nq; q += NT) {
                    const int p = q >= nq, e = q - p * nq;
                    const int i = e >> lq, j = (e & ((G.TW >> 2) - 1)) * 4;
                    *reinterpret_cast<uint32_t*>(&px(k.cur.pl[1 + p], G.baseX + G.TX0 + j, G.baseY + G.TY0 + i)) =
                        *reinterpret_cast<const uint32_t*>(&L.tile[p * C2_TILE + i * TS + j]);
                }
                il_sync<NT>();
                trace_stamp(tr, 9);
                trace_stamp(tr, 10);
                break;
            }
        }
        {
            int r = 0;
            for (int yy = 0; yy < G.ph; yy += G.predH) {
                int c = 0;
                for (int xx = 0; xx < G.pw; xx += G.predW) {
                    const int ix0 = imax(xx, G.TX0), ix1 = imin(xx + G.predW, G.TX0 + G.TW);
                    const int iy0 = imax(yy, G.TY0), iy1 = imin(yy + G.predH, G.TY0 + G.TH);
                    if (ix0 < ix1 && iy0 < iy1)
                        predict_pu<NT, TSZ>(k, blk, L, plane, G.baseX + xx, G.baseY + yy, G.predW, G.predH, G.candRow + r,
                            G.candCol + c, ix0 - xx, iy0 - yy, ix1 - ix0, iy1 - iy0, xx - G.TX0, yy - G.TY0, lw);
                    c++;
                }
                r++;
            }
        }
        if (plane == 0) trace_stamp(tr, 12);
        if (blk.motion_mode == AV1R_OBMC_CAUSAL)
            obmc<NT, TSZ>(k, blk, L, plane, G.baseX, G.baseY, G.predW, G.predH, G.TX0, G.TY0, G.TW, G.TH);
        const DevPlane& dst = k.cur.pl[plane];
        if (!(G.TW & 3)) {  // a dword per lane and row quad (x, TX0 multiples of 4)
            const int lq = ilog2p(G.TW >> 2);
            for (int q = t; q < (G.TW * G.TH) >> 2; q += NT) {
                const int i = q >> lq, j = (q & ((G.TW >> 2) - 1)) * 4;
                *reinterpret_cast<uint32_t*>(&px(dst, G.baseX + G.TX0 + j, G.baseY + G.TY0 + i)) =
                    *reinterpret_cast<const uint32_t*>(&L.tile[i * TSZ + j]);
            }
        } else {
            const int lw = ilog2p(G.TW);
            for (int q = t; q < G.TW * G.TH; q += NT) {
                const int i = q >> lw, j = q & (G.TW - 1);
                px(dst, G.baseX + G.TX0 + j, G.baseY + G.TY0 + i) = L.tile[i * TSZ + j];
            }
        }
        il_sync<NT>();
        trace_stamp(tr, 8 + plane);
    }
}

// Inter-intra blend of block `bi` (Block.cpp:118-144 + maskBlend, InterPredict.cpp:555-609):
// the block's intra prediction (its edges are final when this item runs) blended with the
// inter prediction inter_tile stored in the frame.
template <int NT, bool COH>
DEV void ii_item(const KParams& k, uint32_t bi, TbLds<64>& L, const GranEdges* G = nullptr, bool gran = false,
    const DevBlock* pre = nullptr)
{
    const int t = coop_lane<NT>();
    const DevBlock& blk = pre ? *pre : k.blocks[bi];  // (k_flow: loaded before the wait)
    const int hasChroma = (blk.flags & AV1R_BLK_HAS_CHROMA) != 0;
    const int bs = blk.mi_size;
    const int im = blk.interintra_mode;
    const int isWedge = blk.compound_type == AV1R_COMPOUND_WEDGE;
    WedgeSel ws = {0, 0, 0, 0};
    if (isWedge) ws = wedge_select(bs, blk.wedge_index);
    for (int plane = 0; plane < 1 + hasChroma * 2; plane++) {
        const int psz = plane_bsize(bs, plane);
        const int sub = plane ? 1 : 0;
        const int baseX = (blk.mi_col >> sub) * 4, baseY = (blk.mi_row >> sub) * 4;
        const int pw = av1r_num4x4w[psz] * 4, ph = av1r_num4x4h[psz] * 4;
        const DevPlane& dst = k.cur.pl[plane];
        IntraParams P;
        P.plane = plane;
        P.x = baseX;
        P.y = baseY;
        P.log2W = 2 + av1r_miw_log2[psz];
        P.log2H = 2 + av1r_mih_log2[psz];
        P.haveLeft = plane ? (blk.flags & AV1R_BLK_AVAIL_L_UV) != 0 : (blk.flags & AV1R_BLK_AVAIL_L) != 0;
        P.haveAbove = plane ? (blk.flags & AV1R_BLK_AVAIL_U_UV) != 0 : (blk.flags & AV1R_BLK_AVAIL_U) != 0;
        P.haveAR = (blk.ii_edge >> (2 * plane)) & 1;
        P.haveBL = (blk.ii_edge >> (2 * plane + 1)) & 1;
        P.mode = im == AV1R_II_DC_PRED ? AV1R_DC_PRED : im == AV1R_II_V_PRED ? AV1R_V_PRED
            : im == AV1R_II_H_PRED ? AV1R_H_PRED : AV1R_SMOOTH_PRED;
        P.angleDelta = 0;
        P.filterIntra = 0;
        P.filterIntraMode = 0;
        P.smooth = 0;
        P.edgeFilter = k.hdr->enable_intra_edge_filter;
        if (COH && gran) {  // k_flow with edge granules: G holds plane 0's, 4 mask words per plane
            GranEdges Gp = *G;
            Gp.mask = G->mask + 4 * plane;
            Gp.mA = Gp.mask[0], Gp.mC = Gp.mask[1], Gp.mL = Gp.mask[2];
            Gp.h = k.gran_h[plane];
            Gp.v = k.gran_v[plane];
            Gp.gw = k.gran_w[plane];
            Gp.gh = k.gran_hn[plane];
            coop_intra_edges_gran<NT>(k.mi_cols, k.mi_rows, dst, plane, P.x, P.y, P.log2W, P.log2H, P.haveLeft, P.haveAbove,
                P.haveAR, P.haveBL, L.intra, Gp);
            coop_sync<NT>();
            coop_intra_from_edges<NT>(k.mi_cols, k.mi_rows, P, L.intra, L.pred, 64);
        } else {
            coop_intra_predict<NT, COH>(k.mi_cols, k.mi_rows, dst, P, L.intra, L.pred, 64);
        }
        const int sizeScale = 128 / imax(ph, pw);
        const bool addRes = COH;  // k_flow: the block's residuals are added here (tiles)
        const int lpw = ilog2p(pw);
        for (int q = t; q < pw * ph; q += NT) {
            const int i = q >> lpw, j = q & (pw - 1);
            int m;
            if (!isWedge) {
                m = im == AV1R_II_V_PRED ? av1r_ii_weights_1d[i * sizeScale]
                    : im == AV1R_II_H_PRED ? av1r_ii_weights_1d[j * sizeScale]
                    : im == AV1R_II_SMOOTH_PRED ? av1r_ii_weights_1d[imin(i, j) * sizeScale] : 32;
            } else if (!sub) {
                int mv = wedge_master(ws.dir, ws.yoff + i, ws.xoff + j);
                m = blk.wedge_sign == ws.flip ? mv : 64 - mv;
            } else {
                int s4 = 0;
#pragma unroll
                for (int dy = 0; dy < 2; dy++)
#pragma unroll
                    for (int dx = 0; dx < 2; dx++) {
                        int mw = wedge_master(ws.dir, ws.yoff + 2 * i + dy, ws.xoff + 2 * j + dx);
                        s4 += blk.wedge_sign == ws.flip ? mw : 64 - mw;
                    }
                m = r2(s4, 2);
            }
            const int d = ldp<COH>(dst, baseX + j, baseY + i);  // (flow read site: k_inter's output, final before the launch)
            const uint8_t v = (uint8_t)clip1(r2(m * L.pred[i * 64 + j] + (64 - m) * d, 6));
            if (addRes) L.pred[i * 64 + j] = v;
            else stp<COH>(dst, baseX + j, baseY + i, v);
        }
        coop_sync<NT>();
        if (addRes) {
            // TransformBlock::decode's add and clip for this plane's TBs with coefficients
            // (TBs never overlap: in place in L.pred), then the whole plane is stored
            const int32_t* ext = k.bext + 8 * (size_t)blk.palette_off;
            const uint32_t firstTb = (uint32_t)ext[6], nTbs = (uint32_t)ext[7];
            for (uint32_t ti = firstTb; ti < firstTb + nTbs; ti++) {
                const DevTb& tb = k.tbs[ti];
                if (tb.plane != plane || !tb.coef_cnt) continue;
                const int tw = av1r_tx_w[tb.tx_size], th = av1r_tx_h[tb.tx_size];
                const int16_t* rt = k.res + k.tb_res[ti];
                const int ltw = ilog2p(tw);
                for (int q = t; q < tw * th; q += NT) {
                    const int i = q >> ltw, j = q & (tw - 1);
                    uint8_t& v = L.pred[(tb.y - baseY + i) * 64 + tb.x - baseX + j];
                    v = (uint8_t)clip1(v + rt[q]);
                }
                coop_sync<NT>();
            }
            const bool coh = COH;
            for (int q = t; q < pw * ph; q += NT) {
                const int i = q >> lpw, j = q & (pw - 1);
                stp_c(dst, baseX + j, baseY + i, L.pred[i * 64 + j], coh);
            }
            if (COH && gran)
                coop_publish_gran<NT>(L.pred, 64, baseX, baseY, pw, ph, k.gran_h[plane], k.gran_v[plane], k.gran_w[plane],
                    k.gran_hn[plane], G->epoch);
            coop_sync<NT>();
        }
    }
}

// ---------------------------------------------------------------------------------
// One launch per dependency level: every work item of the level (inter tiles, inter-
// intra blends, transform blocks) is one 64-lane workgroup.
// ---------------------------------------------------------------------------------
// recon.hip is compiled twice (native.py): the level kernels (k_inter, k_tb), and with
// -DAV1R_FLOW_PART k_flow alone -- built without machine-level loop-invariant hoisting,
// which in its persistent loop keeps ~50 constants in VGPRs (177 instead of 124 VGPRs:
// half the occupancy) but which k_inter's pixel loops want.  Each object has its own
// constant-memory parameter table.
#define TB_SMALL 16  // the largest TB side handled one per wave (k_tb, k_flow)

#ifndef AV1R_FLOW_PART
// Level table of one launch over n frames (tab[0..n]: prefix sums of the frames' item
// counts; tab[n + 1 + s]: offset of frame s's items in its item list).  `lane` indexes the
// table (one lane per frame); item `b` of the launch.  Returns the frame's parameters.
DEV const WorkItem& table_item(const KParams* kps, const uint32_t* __restrict__ tab, int n, uint32_t b, const KParams*& kp,
    int& s)
{
    // frame of item b: the number of frames whose items all precede it (one vector load
    // of the prefix table + a ballot instead of a dependent scan)
    const int lane = threadIdx.x & 63;
    const uint32_t pre = lane + 1 < n ? tab[lane + 1] : 0xffffffffu;
    s = __builtin_amdgcn_readfirstlane(__popcll(__ballot(b >= pre)));
    kp = &KP(kps, s);
    return kp->items[tab[n + 1 + s] + (b - tab[s])];
}

// Transform blocks and inter-intra blends of one level.  Large items (a side of 32 or
// more, and the blends) take a whole 256-lane workgroup each; small TBs (up to 16x16) are
// packed four per workgroup, one per wave, each wave with its own small LDS tiles.
// tab: [big prefix (n + 1)][small prefix (n + 1)][big offsets (n)][small offsets (n)].
extern "C" __global__ __launch_bounds__(256) void k_tb(const KParams* kps, const uint32_t* __restrict__ tab, int n,
    unsigned long long* trace, uint32_t traceBase)
{
    constexpr size_t kLds = sizeof(TbLds<64>) > 4 * sizeof(TbLds<TB_SMALL>) ? sizeof(TbLds<64>) : 4 * sizeof(TbLds<TB_SMALL>);
    __shared__ __align__(16) uint8_t smem[kLds];
    const uint32_t* tabS = tab + n + 1;  // small prefix
    const uint32_t nBig = tab[n], nSmall = tabS[n];
    const uint32_t b = xcd_order(blockIdx.x, gridDim.x);
    const KParams* kp;
    int s;
    if (b < nBig) {
        // big: a whole workgroup; offsets follow both prefix tables
        const int lane = threadIdx.x & 63;
        const uint32_t pre = lane + 1 < n ? tab[lane + 1] : 0xffffffffu;
        s = __builtin_amdgcn_readfirstlane(__popcll(__ballot(b >= pre)));
        kp = &KP(kps, s);
        const WorkItem& wi = kp->items[tab[2 * n + 2 + s] + (b - tab[s])];
#ifdef AV1R_TRACE
        unsigned long long* tr = trace ? trace + (size_t)(traceBase + b) * AV1R_TRACE_W : nullptr;
        if (tr && threadIdx.x == 0) {
            tr[0] = wi.code;
            tr[1] = ((unsigned long long)s << 32) | ((unsigned)wi.tx_size << 8) | wi.pred;
        }
#else
        unsigned long long* tr = nullptr;
#endif
        trace_stamp(tr, 2);  // (after the item record: entry and record stamps coincide)
        trace_stamp(tr, 3);
        TbLds<64>& L = *reinterpret_cast<TbLds<64>*>(smem);
        if (AV1R_ITEM_KIND(wi.code) == AV1R_ITEM_II) ii_item<256, false>(*kp, AV1R_ITEM_INDEX(wi.code), L);
        else tb_item<256, 64>(*kp, wi, L, tr);
        trace_stamp(tr, 5);
        return;
    }
    // small: item i of the small list, one per wave
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (uniform: a wave past the list returns as a whole)
    const uint32_t i = (b - nBig) * 4 + wave;
    if (i >= nSmall) return;  // (no workgroup barrier in this mode)
    const int lane = threadIdx.x & 63;
    const uint32_t pre = lane + 1 < n ? tabS[lane + 1] : 0xffffffffu;
    s = __builtin_amdgcn_readfirstlane(__popcll(__ballot(i >= pre)));
    kp = &KP(kps, s);
    const WorkItem& wi = kp->items[tab[3 * n + 2 + s] + (i - tabS[s])];
#ifdef AV1R_TRACE
    unsigned long long* tr = trace ? trace + (size_t)(traceBase + nBig + i) * AV1R_TRACE_W : nullptr;
    if (tr && lane == 0) {
        tr[0] = wi.code;
        tr[1] = ((unsigned long long)s << 32) | ((unsigned)wi.tx_size << 8) | wi.pred;
    }
#else
    unsigned long long* tr = nullptr;
    (void)trace;
    (void)traceBase;
#endif
    trace_stamp(tr, 2);
    trace_stamp(tr, 3);
    TbLds<TB_SMALL>& L = reinterpret_cast<TbLds<TB_SMALL>*>(smem)[wave];
    tb_item<64, TB_SMALL>(*kp, wi, L, tr);
    trace_stamp(tr, 5);
}

// 4 waves/SIMD (128 VGPRs, 64 B/lane of spills; LDS 10160 B: 16 workgroups/CU); the
// -DAV1R_TRACE build keeps its registers (with the stamps it would spill ~1.9 KB/lane)
#ifndef AV1R_INTER_WAVES
#define AV1R_INTER_WAVES 3  // 3 waves/SIMD: 163 VGPRs, no spills (4: 128 VGPRs + 88 B/lane scratch, no faster, 2x the HBM writes)
#endif
#if defined(AV1R_TRACE) || AV1R_INTER_WAVES == 0
#define K_INTER_BOUNDS __launch_bounds__(64)
#else
#define K_INTER_BOUNDS __launch_bounds__(64, AV1R_INTER_WAVES)
#endif
DEV void inter_general(const KParams* kps, const uint32_t* __restrict__ tab, int n, uint32_t b, InterLds& L,
    unsigned long long* trace, uint32_t traceBase)
{
    const unsigned long long tEntry = trace ? trace_now() : 0;
    const KParams* kp;
    int s;
    // the tile's code (frame of tile b: the number of frames whose tiles all precede it)
    const int lane = threadIdx.x & 63;
    const uint32_t pre = lane + 1 < n ? tab[lane + 1] : 0xffffffffu;
    s = __builtin_amdgcn_readfirstlane(__popcll(__ballot(b >= pre)));
    kp = &KP(kps, s);
    const uint32_t pos = tab[n + 1 + s] + (b - tab[s]);
    const uint32_t code = sload(kp->tiles + pos);
    const uint32_t idx = AV1R_ITEM_INDEX(code);
#ifdef AV1R_TRACE
    // traceBase ~0u (k_flow mode): frame-major rows, this frame's base + its items + the tile position
    const size_t row = traceBase == ~0u ? kp->trace_base + kp->n_items + pos : (size_t)traceBase + b;
    unsigned long long* tr = trace ? trace + row * AV1R_TRACE_W : nullptr;
#else
    unsigned long long* tr = nullptr;
    (void)trace;
    (void)traceBase;
#endif
    trace_put(tr, 2, tEntry);
    trace_put(tr, 0, code);
    trace_stamp(tr, 3);
    inter_tile<64, TS>(*kp, idx >> 4, idx & 3, (idx >> 2) & 3, L, tr);
    trace_stamp(tr, 5);
}
extern "C" __global__ K_INTER_BOUNDS void k_inter(const KParams* kps, const uint32_t* __restrict__ tab, int n,
    unsigned long long* trace, uint32_t traceBase)
{
    __shared__ __align__(16) InterLds L;
    inter_general(kps, tab, n, xcd_order(blockIdx.x, gridDim.x), L, trace, traceBase);
}

// ---------------------------------------------------------------------------------
// k_inter_s / k_inter_m: small / medium plain inter blocks, four / two per wave.
//
// Blocks with both luma sides <= 8 are most of an inter frame's tiles, and k_inter gives
// each a whole wave (and its 128-VGPR register budget for every prediction mode) while
// its 8x8 luma needs 16 lanes.  The plain ones (simple motion, single reference or
// average / distance compound, unwarped, unscaled: classified by the host, build_schedule)
// go to k_inter_s instead: 16 lanes per block, the unit's state per lane, ~1 KB of LDS
// each, the samples stored straight to the frame -- many more blocks in flight per CU.
// Plain blocks with both sides <= 16 go to k_inter_m the same way, 32 lanes each.
// ---------------------------------------------------------------------------------
template <int MS>
struct SmallLds {
    uint8_t win[2][(MS + 7) * (MS + 8)];  // reference windows: <= MS + 7 rows, stride MS + 8
    int16_t hb[2][(MS + 7) * MS];         // their horizontally filtered rows
};

// One prediction unit (predict_inter, InterPredict.cpp:962-1049; blockInterPrediction's
// sub-pel filter, :319-383; the average / distance blend of :1022-1049) of w x h <= 8 x 8
// at plane position (x, y), by NT lanes.
template <int NT, int MS>
DEV void small_pu(const KParams& k, SmallLds<MS>& L, const DevBlock& blk, int plane, int x, int y, int w, int h, int candRow,
    int candCol)
{
    const int t = threadIdx.x & (NT - 1);
    const int ct = blk.compound_type;
    const PuInfo info = pu_info(k, blk, candRow, candCol);
    const int isCompound = info.ref_frame[1] > AV1R_INTRA_FRAME;
    uint2 hf[2];
    uint4 vf[2];
    int integer[2] = {1, 1};
#pragma unroll
    for (int l = 0; l < 2; l++) {
        if (l > isCompound) break;
        RefSel R;
        select_ref(k, R, k.hdr->ref_frame_idx[info.ref_frame[l] - 1], plane, x, y, info.mv[l]);
        const int fx = filter_idx(info.filt, w, 1), fy = filter_idx(info.filt, h, 0);
        const int hph = (R.startX >> 6) & 15, vph = (R.startY >> 6) & 15;
        integer[l] = !hph && !vph;
        hf[l] = hfilt_pk(fx * 16 + hph);
        vf[l] = vfilt_pk(fy * 16 + vph);
        load_window<NT, MS>(R, L.win[l], 0, 0, w, h, MS + 8);
    }
    coop_sync<NT>();
#pragma unroll
    for (int l = 0; l < 2; l++)
        if (l <= isCompound && !integer[l]) hpass<NT>(L.win[l], L.hb[l], w, h, hf[l], 3, MS + 8, MS);
    coop_sync<NT>();
    const int R1 = isCompound ? 7 : 11, PostRound = 14 - (3 + R1);
    int fwd = 0, bck = 0;
    const int dist = isCompound && ct == AV1R_COMPOUND_DISTANCE;
    if (dist) distance_weights(k, info, fwd, bck);
    auto blend = [&](int p0, int p1) {
        return !isCompound ? clip1(p0)
             : dist        ? clip1(r2(fwd * p0 + bck * p1, 4 + PostRound))
                           : clip1(r2(p0 + p1, 1 + PostRound));
    };
    const DevPlane& dst = k.cur.pl[plane];
    if (!(w & 3)) {
        const int g4 = w >> 2, lg = ilog2p(g4);  // (w: a power of two)
        for (int q = t; q < h * g4; q += NT) {
            const int rr = q >> lg, cc = (q & (g4 - 1)) * 4;
            int p0[4], p1[4] = {0, 0, 0, 0};
            pred_win4(L.win[0], L.hb[0], rr, cc, 3, R1, vf[0], integer[0], p0, MS + 8, MS);
            if (isCompound) pred_win4(L.win[1], L.hb[1], rr, cc, 3, R1, vf[1], integer[1], p1, MS + 8, MS);
            uint32_t v = 0;
#pragma unroll
            for (int m = 0; m < 4; m++) v |= (uint32_t)blend(p0[m], p1[m]) << (8 * m);
            *reinterpret_cast<uint32_t*>(&px(dst, x + cc, y + rr)) = v;  // x, cc: multiples of 4
        }
    } else {
        const int lw = ilog2p(w);
        for (int q = t; q < h * w; q += NT) {
            const int rr = q >> lw, cc = q & (w - 1);
            const int p0 = pred_win(L.win[0], L.hb[0], rr, cc, 3, R1, vf[0], integer[0], MS + 8, MS);
            const int p1 = isCompound ? pred_win(L.win[1], L.hb[1], rr, cc, 3, R1, vf[1], integer[1], MS + 8, MS) : 0;
            px(dst, x + cc, y + rr) = (uint8_t)blend(p0, p1);
        }
    }
    coop_sync<NT>();  // the next unit reuses the windows
}

// Both chroma planes of a block whose chroma is ONE prediction unit (the usual case): U and V
// share the unit's motion, filters and window geometry, so their windows -- two planes x up
// to two references -- go out in one memory round trip (per plane, small_pu costs one each),
// then the passes run over both.  The windows and intermediates are laid over the group's
// SmallLds (4 windows of (MS/2 + 7) x (MS/2 + 8) bytes, then 4 intermediates).
template <int NT, int MS>
DEV void small_pu_c2(const KParams& k, SmallLds<MS>& L, const DevBlock& blk, int x, int y, int w, int h, int candRow,
    int candCol)
{
    constexpr int CS = MS / 2, WS = CS + 8, WSZ = (CS + 7) * WS, HSZ = (CS + 7) * CS;
    constexpr int WALL = (4 * WSZ + 7) & ~7;
    static_assert(WALL + 4 * HSZ * 2 <= sizeof(SmallLds<MS>), "chroma pair windows exceed the group's LDS");
    uint8_t* win = reinterpret_cast<uint8_t*>(&L);
    int16_t* hb = reinterpret_cast<int16_t*>(win + WALL);
    const int t = threadIdx.x & (NT - 1);
    const int ct = blk.compound_type;
    const PuInfo info = pu_info(k, blk, candRow, candCol);
    const int isCompound = info.ref_frame[1] > AV1R_INTRA_FRAME;
    uint2 hf[2];
    uint4 vf[2];
    int integer[2] = {1, 1};
#pragma unroll
    for (int l = 0; l < 2; l++) {
        if (l > isCompound) break;
        const int slot = k.hdr->ref_frame_idx[info.ref_frame[l] - 1];
        RefSel R;
        select_ref(k, R, slot, 1, x, y, info.mv[l]);
        const int fx = filter_idx(info.filt, w, 1), fy = filter_idx(info.filt, h, 0);
        const int hph = (R.startX >> 6) & 15, vph = (R.startY >> 6) & 15;
        integer[l] = !hph && !vph;
        hf[l] = hfilt_pk(fx * 16 + hph);
        vf[l] = vfilt_pk(fy * 16 + vph);
        load_window<NT, CS>(R, win + l * WSZ, 0, 0, w, h, WS);
        R.p = k.ref[slot].pl[2];  // V: the same extent as U
        load_window<NT, CS>(R, win + (2 + l) * WSZ, 0, 0, w, h, WS);
    }
    coop_sync<NT>();
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int l = q & 1;
        if (l <= isCompound && !integer[l]) hpass<NT>(win + q * WSZ, hb + q * HSZ, w, h, hf[l], 3, WS, CS);
    }
    coop_sync<NT>();
    const int R1 = isCompound ? 7 : 11, PostRound = 14 - (3 + R1);
    int fwd = 0, bck = 0;
    const int dist = isCompound && ct == AV1R_COMPOUND_DISTANCE;
    if (dist) distance_weights(k, info, fwd, bck);
    auto blend = [&](int p0, int p1) {
        return !isCompound ? clip1(p0)
             : dist        ? clip1(r2(fwd * p0 + bck * p1, 4 + PostRound))
                           : clip1(r2(p0 + p1, 1 + PostRound));
    };
#pragma unroll
    for (int p = 0; p < 2; p++) {
        const DevPlane& dst = k.cur.pl[1 + p];
        const uint8_t* w0 = win + (2 * p) * WSZ;
        const uint8_t* w1 = win + (2 * p + 1) * WSZ;
        const int16_t* h0 = hb + (2 * p) * HSZ;
        const int16_t* h1 = hb + (2 * p + 1) * HSZ;
        if (!(w & 3)) {
            const int g4 = w >> 2, lg = ilog2p(g4);
            for (int q = t; q < h * g4; q += NT) {
                const int rr = q >> lg, cc = (q & (g4 - 1)) * 4;
                int p0[4], p1[4] = {0, 0, 0, 0};
                pred_win4(w0, h0, rr, cc, 3, R1, vf[0], integer[0], p0, WS, CS);
                if (isCompound) pred_win4(w1, h1, rr, cc, 3, R1, vf[1], integer[1], p1, WS, CS);
                uint32_t v = 0;
#pragma unroll
                for (int m = 0; m < 4; m++) v |= (uint32_t)blend(p0[m], p1[m]) << (8 * m);
                *reinterpret_cast<uint32_t*>(&px(dst, x + cc, y + rr)) = v;
            }
        } else {
            const int lw = ilog2p(w);
            for (int q = t; q < h * w; q += NT) {
                const int rr = q >> lw, cc = q & (w - 1);
                const int p0 = pred_win(w0, h0, rr, cc, 3, R1, vf[0], integer[0], WS, CS);
                const int p1 = isCompound ? pred_win(w1, h1, rr, cc, 3, R1, vf[1], integer[1], WS, CS) : 0;
                px(dst, x + cc, y + rr) = (uint8_t)blend(p0, p1);
            }
        }
    }
    coop_sync<NT>();  // the next block's units reuse the LDS
}

// Frames' lists are dealt in groups of 64 / NT (a frame's last group may be partial), so
// the parameters of a workgroup stay uniform.  tab: [group prefix (n + 1)][offsets (n)][counts (n)].
template <int NT, int MS>
DEV void inter_plain(const KParams* kps, const uint32_t* __restrict__ tab, int n, uint32_t b, SmallLds<MS>* L)
{
    const int lane = threadIdx.x & 63;
    const uint32_t pre = lane + 1 < n ? tab[lane + 1] : 0xffffffffu;
    const int s = __builtin_amdgcn_readfirstlane(__popcll(__ballot(b >= pre)));
    const KParams& k = KP(kps, s);
    const int g = threadIdx.x / NT;
    const uint32_t i = (64 / NT) * (b - tab[s]) + g;
    if (i >= tab[2 * n + 1 + s]) return;  // (wave-level ordering only: no barrier follows)
    const DevBlock& blk = k.blocks[AV1R_ITEM_INDEX(k.tiles[tab[n + 1 + s] + i]) >> 4];
    const int nPl = (blk.flags & AV1R_BLK_HAS_CHROMA) ? 3 : 1;
    for (int plane = 0; plane < nPl; plane++) {
        // (sub-8x8 chroma may gather up to four units of neighbouring blocks)
        const PlaneGeo G = plane_geo<MS>(k, blk, plane, 0, 0);
        // (a block whose chroma is one prediction unit: both planes' windows in one memory
        // round trip -- round 5: 0.0484 -> 0.0480 ms/frame, kept)
        if (plane == 1 && G.predW == G.pw && G.predH == G.ph && G.candRow == blk.mi_row && G.candCol == blk.mi_col) {
            small_pu_c2<NT, MS>(k, L[g], blk, G.baseX, G.baseY, G.pw, G.ph, G.candRow, G.candCol);
            break;
        }
        int r = 0;
        for (int yy = 0; yy < G.ph; yy += G.predH, r++) {
            int c = 0;
            for (int xx = 0; xx < G.pw; xx += G.predW, c++)
                small_pu<NT, MS>(k, L[g], blk, plane, G.baseX + xx, G.baseY + yy, G.predW, G.predH, G.candRow + r,
                    G.candCol + c);
        }
    }
}
#ifndef AV1R_PLAIN_WAVES
#define AV1R_PLAIN_WAVES 0  // minimum waves/SIMD for k_inter_s / k_inter_m (0: the compiler's choice, 153 VGPRs = 3)
#endif
#if AV1R_PLAIN_WAVES
#define K_PLAIN_BOUNDS __launch_bounds__(64, AV1R_PLAIN_WAVES)
#else
#define K_PLAIN_BOUNDS __launch_bounds__(64)
#endif
extern "C" __global__ K_PLAIN_BOUNDS void k_inter_s(const KParams* kps, const uint32_t* __restrict__ tab, int n)
{
    __shared__ SmallLds<8> L[4];
    inter_plain<16, 8>(kps, tab, n, xcd_order(blockIdx.x, gridDim.x), L);
}
extern "C" __global__ K_PLAIN_BOUNDS void k_inter_m(const KParams* kps, const uint32_t* __restrict__ tab, int n)
{
    __shared__ SmallLds<16> L[2];
    inter_plain<32, 16>(kps, tab, n, xcd_order(blockIdx.x, gridDim.x), L);
}

// All inter tiles of a launch in ONE grid (the dataflow schedule's level 0): the general
// tiles (k_inter: warps, OBMC, masked compounds, scaled references, larger blocks), then the
// medium and the small plain blocks (k_inter_m / k_inter_s), as three kernels one after the
// other left each one's tail of idle CUs before the next could start.  Every class count is
// padded to a multiple of 8 (padding workgroups return at once), and XCD x (blockIdx % 8, as
// the hardware deals workgroups) runs the x-th contiguous eighth of each class in class order:
// each XCD takes its share of the long general tiles first, and a frame's tiles of one class
// stay on one XCD's L2 (as xcd_order gives each kernel).  Placement is a speed heuristic only:
// every logical index is run by exactly one workgroup wherever it lands.
// tab: [k_inter table][k_inter_m table][k_inter_s table] (launch_jobs); gI / gM / gS the classes'
// padded workgroup counts.
// Each class is cut into 8 contiguous eighths, eighth x to XCD x (round 5: several chunks per
// XCD, mixing frames' regions into each share, measured within noise,
// profiles/r05_ab_xcd_dealing.txt).  The class counts are padded to multiples of 8 * bands.
DEV uint32_t inter_deal(uint32_t x, uint32_t j, uint32_t q)
{
    return x * q + j;
}
extern "C" __global__ K_INTER_BOUNDS void k_inter_all(const KParams* kps, const uint32_t* __restrict__ tab, int n,
    uint32_t gI, uint32_t gM, uint32_t gS, uint32_t nb, unsigned long long* trace)
{
    union Lds {
        InterLds g;
        SmallLds<16> m[2];
        SmallLds<8> s[4];
    };
    __shared__ __align__(16) Lds L;
    const uint32_t x = blockIdx.x & 7, j = blockIdx.x >> 3;
    const uint32_t qI = gI >> 3, qM = gM >> 3, qS = gS >> 3;
    const uint32_t* tI = tab;
    const uint32_t* tM = tI + 2 * n + 1;
    const uint32_t* tS = tM + 3 * n + 1;
    // nb: bands (AV1R_INTER_BANDS): with nb > 1 each XCD walks its share band by band -- the
    // general, medium and small tiles of band 0, then of band 1, ... (the class lists are in
    // decode order, so a band is a stretch of the frame) -- so that a region's reference lines
    // are fetched once for all three classes, not once per class sweep.  The class counts are
    // padded to multiples of 8 * bands.
    uint32_t cls = 3, jj = 0;
    if (nb == 1) {
        if (j < qI) cls = 0, jj = j;
        else if (j < qI + qM) cls = 1, jj = j - qI;
        else if (j < qI + qM + qS) cls = 2, jj = j - qI - qM;
    } else {
        const uint32_t bI = qI / nb, bM = qM / nb, bS = qS / nb, per = bI + bM + bS;
        const uint32_t band = j / per, r = j - band * per;
        if (band < nb) {
            if (r < bI) cls = 0, jj = band * bI + r;
            else if (r < bI + bM) cls = 1, jj = band * bM + (r - bI);
            else cls = 2, jj = band * bS + (r - bI - bM);
        }
    }
    if (cls == 0) {
        const uint32_t b = inter_deal(x, jj, qI);
        if (b < tI[n]) inter_general(kps, tI, n, b, L.g, trace, ~0u);
    } else if (cls == 1) {
        const uint32_t b = inter_deal(x, jj, qM);
        if (b < tM[n]) inter_plain<32, 16>(kps, tM, n, b, L.m);
    } else if (cls == 2) {
        const uint32_t b = inter_deal(x, jj, qS);
        if (b < tS[n]) inter_plain<16, 8>(kps, tS, n, b, L.s);
    }
}

#endif  // !AV1R_FLOW_PART

#ifdef AV1R_FLOW_PART
// ---------------------------------------------------------------------------------
// k_flow: all transform-block and inter-intra items of a batch in ONE persistent launch,
// ordered by their data dependencies instead of by one launch per level.
//
// The host lists the items' groups (one large item, or up to four small ones: the same
// packing as k_tb) in a topological order: level by level, frames interleaved.  Group g
// belongs to queue g % 8; the k-th workgroup to START serves queue k % 8 and pulls its
// next group with one atomic add, so a queue's groups are taken in order.  Every item
// waits only for items of EARLIER groups (its dependency list, built by the host from the
// 4x4 units whose pixels it reads: intra edges, CFL luma, the inter-intra prediction), so
// the earliest unfinished group is either held by a running workgroup whose dependencies
// are all complete, or is the next group of a queue whose workgroups are all free.  A
// workgroup leaves only when its queue has no group left to hand out, so once 8 of the
// grid's workgroups have started every queue with work has a resident server: the launch
// progresses whatever the residency or placement.  Several overlapping k_flow grids (from
// different streams) cannot starve each other either: they never wait on one another, so
// while the chip holds >= 8 workgroups of some grid that grid finishes and frees its
// slots (1536 slots at 6 per CU: up to 192 overlapping grids).
//
// Hand-off between items (cdna_hip_programming.md §6 Guideline 16, R1): a producer stores
// its pixels write-through (stp/stp4<true>: sc1), every storing wave drains them
// (s_waitcnt vmcnt(0)), then one lane stores the item's done word = the launch's epoch
// (sc1).  A consumer polls its dependencies' done words (one lane each, sc1 loads), then
// reads every pixel another item of the launch may have written with sc1 loads (ldp /
// ldp4<true>), which bypass the CU's L1.  The residual of a TB reads only the batch, so it
// is computed BEFORE the wait, off the dependency chain.  Every spin is bounded: after
// FLOW_SPINS polls (or once any wave has timed out) the wave gives up and sets the
// launch's error word, which the host reports.
// ---------------------------------------------------------------------------------

#include "intra_fast.h"

template <int NT>
DEV void flow_wait(const uint32_t* deps, uint32_t nd, const uint32_t* done, uint32_t epoch, uint32_t* ctl)
{
    if (nd && (NT == 64 || threadIdx.x < 64)) {
        const int lane = threadIdx.x & 63;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t spins = 0, lim = 0;
        for (uint32_t b = 0; b < nd; b += 64) {
            const bool mine = b + lane < nd;
            const uint32_t d = mine ? deps[b + lane] : 0u;
            for (;;) {
                const bool ok = !mine || __hip_atomic_load(done + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
                if (__all(ok)) break;
                const bool dead =
                    (spins & AV1R_ERR_POLL_MASK) == 0 && __hip_atomic_load(ctl + FLOW_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                if (!lim) lim = flow_spin_limit(ctl);
                if (dead || ++spins > lim || __builtin_amdgcn_s_memrealtime() - t0 > FLOW_WALL) {
                    if (lane == 0 && !dead) {  // the wave that gave up first reports
                        __hip_atomic_store(ctl + FLOW_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        // the host's copy (pinned memory, checked when the launch's metadata is reused)
                        __hip_atomic_store(reinterpret_cast<uint32_t*>(*reinterpret_cast<uint32_t* const*>(ctl + FLOW_HOSTERR)),
                            1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    b = nd;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
    }
    if (NT > 64) __syncthreads();
    asm volatile("" ::: "memory");  // no pixel load moves above the poll
}

// every storing wave drains its write-through stores, then one lane publishes
template <int NT>
DEV void flow_publish(uint32_t* flag, uint32_t epoch)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (NT > 64) __syncthreads();
    if (coop_lane<NT>() == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// -DAV1R_TRACE timeline row (frame-major): 0 code, 1 frame << 32 | tx_size << 8 | pred,
// 2 entry, 3 residual done, 4 dependencies complete, 5 published, 6 level (host),
// 7 XCC id << 16 | dependency count
template <int NT, int MAX>
DEV void flow_item(const KParams& k, uint32_t pos, TbLds<MAX>& L, uint32_t epoch, uint32_t* ctl,
    unsigned long long* trace, uint32_t s)
{
    // What the item reads from the batch after its wait -- its edge mask words, its block's
    // prediction fields, the edge-filter flag (and with AV1R_FLOW_ITEM_COPY its own record)
    // -- is loaded into registers BEFORE the wait: after it (the wait's memory clobber
    // forces a reload) each was one more dependent round trip on every hop of the chain.
#ifndef AV1R_FLOW_ITEM_COPY
#define AV1R_FLOW_ITEM_COPY 1  // k_flow -9 %, device-only +5 % (A/B on one box; costs 16 B/lane of scratch)
#endif
#if AV1R_FLOW_ITEM_COPY
    const WorkItem wi = sload(k.items + pos);  // (scalar registers, live across the wait)
#else
    const WorkItem& wi = k.items[pos];
#endif
#ifdef AV1R_TRACE
    unsigned long long* tr = trace ? trace + (size_t)(k.trace_base + pos) * AV1R_TRACE_W : nullptr;
    trace_stamp(tr, 2);
    trace_put(tr, 0, wi.code);
    trace_put(tr, 1, ((unsigned long long)s << 32) | ((unsigned)wi.tx_size << 8) | wi.pred);
    // (HW_ID in the upper half: wave, SIMD, CU, SH, SE of the wave -- tools/trace_run.py's
    // per-slot occupancy)
    trace_put(tr, 7, ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) << 32) |
                         ((unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 16) | wi.dep_cnt);
#else
    unsigned long long* tr = nullptr;
    (void)trace;
    (void)s;
#endif
    // edge granules: the item's mask words precede its dependency list (4 per plane)
    // (G goes to the predictors by address whatever `gran` says: a pointer that is either
    // &G or null made G a 64 B/lane stack object -- scratch traffic on every item)
    const bool gran = k.gran;
    GranEdges G = {};
    uint32_t resOff = ~0u;  // a TB's residual tile: the fourth mask word (granules), else tb_res
    if (gran) {
        const int p = AV1R_ITEM_KIND(wi.code) == AV1R_ITEM_II ? 0 : wi.plane;
        G.mask = k.deps + wi.dep_off - (AV1R_ITEM_KIND(wi.code) == AV1R_ITEM_II ? 12 : 4);
        const uint4 m4 = sload(reinterpret_cast<const uint4*>(G.mask));
        G.mA = m4.x, G.mC = m4.y, G.mL = m4.z;
        resOff = m4.w;
        G.h = k.gran_h[p];
        G.v = k.gran_v[p];
        G.gw = k.gran_w[p];
        G.gh = k.gran_hn[p];
        G.epoch = epoch;
        G.ctl = ctl;
        G.coh = true;
        G.tr = tr;
    }
    if (AV1R_ITEM_KIND(wi.code) == AV1R_ITEM_II) {
        if constexpr (MAX == 64) {  // blends are always large items
            const DevBlock blk = sload(k.blocks + AV1R_ITEM_INDEX(wi.code));
            trace_stamp(tr, 3);
            flow_wait<NT>(k.deps + wi.dep_off, wi.dep_cnt, k.done, epoch, ctl);
            trace_stamp(tr, 4);
            ii_item<NT, true>(k, AV1R_ITEM_INDEX(wi.code), L, &G, gran, &blk);
        }
    } else {
        // intra / palette TB: its residual tile (k_resid) is fetched before the wait
        ResQuads<NT, MAX> R;
        if (!gran) resOff = wi.coef_cnt ? sload(k.tb_res + AV1R_ITEM_INDEX(wi.code)) : ~0u;
        res_prefetch<NT, MAX>(k, wi, resOff, R);
        const DevBlock blk = sload(k.blocks + wi.block);  // (a copy: only the fields predict reads are loaded)
        const int edgeFilter = sfield(&k.hdr->enable_intra_edge_filter);
        bool lean = false;
        if constexpr (NT == 64 && MAX == TB_SMALL) {
            // small intra TBs: the lean path (intra_fast.h), its parameters set up before the wait
            if (gran && k.fi && fi_ok(wi, blk)) {
                lean = true;
                const FiParams F = fi_setup(k, wi, blk, edgeFilter);
                trace_stamp(tr, 3);
                flow_wait<NT>(k.deps + wi.dep_off, wi.dep_cnt, k.done, epoch, ctl);
                trace_stamp(tr, 4);
                fi_run<MAX>(k, wi, F, L, G, R.r[0], epoch, gran);
                trace_stamp(tr, 10);
            }
        }
        if (!lean) {
            trace_stamp(tr, 3);
            flow_wait<NT>(k.deps + wi.dep_off, wi.dep_cnt, k.done, epoch, ctl);
            trace_stamp(tr, 4);
            tb_predict<NT, MAX, true>(k, wi, blk, L, &G, gran, edgeFilter);
            trace_stamp(tr, 9);
            tb_store_flow<NT, MAX>(k, wi, L, R, epoch);
            trace_stamp(tr, 10);
        }
    }
    // the store drain and done flag only where a dependency list names the item (CFL's
    // luma; every edge owner without granules): edges travel in granules, and later
    // launches see every store anyway
    if ((wi.pub & 1) || !gran) flow_publish<NT>(k.done + pos, epoch);
    trace_stamp(tr, 5);
    trace_flush(tr);
}

// ---------------------------------------------------------------------------------
// Tiny items (round 6): intra TBs of at most 8x8 on the lean path, four per wave, one per
// 16-lane row (TinyItem, av1r_dev.h).  fi_run (intra_fast.h) runs one item per wave with its
// parameters uniform; an item's time there was load latency -- its record loads, the edge
// gather's round trip, the group's barrier and ticket -- around ~1.7 us of prediction and
// store (profiles/r05_trace_flow_levelorder.txt: 8.8 us of the 10.5 per item), with a 4x4
// TB using 4 of the wave's 64 lanes.  Here the four rows' records arrive in one scalar round
// trip, their residual quads, dependency polls and edge units in one vector round trip
// (+ the polls), and the predictions run side by side: the same arithmetic as fi_run per
// row, with the row's parameters in VGPRs (the rows' classes may differ: divergent).
// Items of one group are of one level, so none waits for another.
// ---------------------------------------------------------------------------------
#define TE_OFF 16
#define TE_LEN (TE_OFF + 48)
struct TinyLds {
    uint8_t above[TE_LEN], left[TE_LEN], upA[TE_LEN], upL[TE_LEN];
    uint32_t ua[4];  // the above run's units (pixel (x + i, y - 1) at byte i)
    uint32_t ul[8];  // the left run's units (pixel (x - 1, y + i) at byte i); [7]: the corner's
};
DEV uint32_t row_sel(int row, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    return row == 0 ? a : row == 1 ? b : row == 2 ? c : d;
}
// the total of v over each 16-lane row, in every lane of the row (fi_row_sum leaves it in
// lane 15; ds_swizzle in bit mode reads lane (l & 0x10) | 0xf of each 32-lane half)
DEV int row16_total(int v)
{
    return __builtin_amdgcn_ds_swizzle(fi_row_sum(v), 0x1F0);
}
DEV uint32_t bits(uint32_t v, int lo, int n) { return (v >> lo) & ((1u << n) - 1); }
// every lane's dependency d (~0u: none) done, as flow_wait (bounded, error word 1)
DEV void flow_wait_lanes(uint32_t d, const uint32_t* done, uint32_t epoch, uint32_t* ctl)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t spins = 0, lim = 0;
    for (;;) {
        const bool ok = d == ~0u || __hip_atomic_load(done + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
        if (__all(ok)) break;
        const bool dead = (spins & AV1R_ERR_POLL_MASK) == 0 && __hip_atomic_load(ctl + FLOW_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        if (!lim) lim = flow_spin_limit(ctl);
        if (dead || ++spins > lim || __builtin_amdgcn_s_memrealtime() - t0 > FLOW_WALL) {
            if ((threadIdx.x & 63) == 0 && !dead) {
                __hip_atomic_store(ctl + FLOW_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(reinterpret_cast<uint32_t*>(*reinterpret_cast<uint32_t* const*>(ctl + FLOW_HOSTERR)), 1u,
                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// -DAV1R_TRACE lite stamps of a tiny item (its row's lane 0 writes its timeline row directly,
// no waits): 2 entry, 3 records in, 4 dependencies and edge units in, 8 units in LDS, 9
// predicted, 10 stored, 5 published; 0 / 1 / 7 as flow_item's
#if defined(AV1R_TRACE) && defined(AV1R_TRACE_LITE)
#define TINY_STAMP(s) \
    if (tr && t == 0) tr[s] = __builtin_amdgcn_s_memrealtime()
#else
#define TINY_STAMP(s) (void)0
#endif
// pos0: the group's first item; nIt: its items (<= 16); T: this wave's four rows
DEV void tiny_run(const KParams& k, uint32_t pos0, uint32_t nIt, TinyLds* T, uint32_t epoch, uint32_t* ctl,
    unsigned long long* trace, uint32_t frame)
{
    const int lane = threadIdx.x & 63, row = lane >> 4;
    int t = lane & 15;
    asm volatile("" : "+v"(t));  // (as coop_lane: no lane-derived address hoisted)
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#if defined(AV1R_TRACE) && defined(AV1R_TRACE_LITE)
    unsigned long long* tr = trace && wave + 4 * row < nIt ? trace + (size_t)(k.trace_base + pos0 + wave + 4 * row) * AV1R_TRACE_W : nullptr;
    TINY_STAMP(2);
    if (tr && t == 0) {
        tr[0] = AV1R_ITEM(AV1R_ITEM_TB, 0);
        tr[1] = (unsigned long long)frame << 32;
        tr[7] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) << 32) |
                ((unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 16);
    }
#else
    (void)trace;
    (void)frame;
#endif
    // ---- the rows' records: four scalar loads, merged per lane
    uint32_t d[8];
    {
        uint32_t s[4][8];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint32_t i = imin(wave + 4 * r, nIt - 1);  // (a row past the group re-reads the last)
            const uint4 a = sload(reinterpret_cast<const uint4*>(k.items + pos0 + i));
            const uint4 b = sload(reinterpret_cast<const uint4*>(k.items + pos0 + i) + 1);
            s[r][0] = a.x, s[r][1] = a.y, s[r][2] = a.z, s[r][3] = a.w;
            s[r][4] = b.x, s[r][5] = b.y, s[r][6] = b.z, s[r][7] = b.w;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) d[j] = row_sel(row, s[0][j], s[1][j], s[2][j], s[3][j]);
    }
    const bool act = wave + 4 * row < nIt;
    const uint32_t pos = pos0 + wave + 4 * row;
    TINY_STAMP(3);
    const int x = (int)(d[0] & 0xffff), y = (int)(d[0] >> 16);
    const int plane = (int)bits(d[1], 0, 2);
    const int log2W = 2 + (int)bits(d[1], 2, 1), log2H = 2 + (int)bits(d[1], 3, 1);
    const int cls = (int)bits(d[1], 4, 4);
    const uint32_t fl = bits(d[1], 8, 8);
    const bool hA = fl & TI_HA, hL = fl & TI_HL, cfl = fl & TI_CFL;
    const int w = 1 << log2W, h = 1 << log2H, w4 = w >> 2;
    const int nq = (w * h) >> 2;  // quads
    const int qi = t >> (log2W - 2), qj = (t & (w4 - 1)) << 2;
    // the row's plane: frame and granule arrays (uniform per plane, selected per lane)
    const DevPlane P0 = k.cur.pl[0], P1 = k.cur.pl[1], P2 = k.cur.pl[2];
    DevPlane dst;
    dst.p = plane == 0 ? P0.p : plane == 1 ? P1.p : P2.p;
    dst.stride = plane == 0 ? P0.stride : plane == 1 ? P1.stride : P2.stride;
    dst.w = dst.h = 0;
    const uint64_t* gh = plane == 0 ? k.gran_h[0] : plane == 1 ? k.gran_h[1] : k.gran_h[2];
    const uint64_t* gv = plane == 0 ? k.gran_v[0] : plane == 1 ? k.gran_v[1] : k.gran_v[2];
    const int gw = plane == 0 ? k.gran_w[0] : plane == 1 ? k.gran_w[1] : k.gran_w[2];
    const int ghn = plane == 0 ? k.gran_hn[0] : plane == 1 ? k.gran_hn[1] : k.gran_hn[2];
    // ---- one round trip: the residual quad, the first 16 dependencies, the edge units (the
    // frame's pixels for units final before the launch, first granule polls for the others)
    const uint32_t resOff = d[7];
    uint2 res = make_uint2(0, 0);
    if (act && resOff != ~0u && t < nq) res = reinterpret_cast<const uint2*>(k.res + resOff)[t];
    const uint32_t depOff = d[5], depCnt = d[6] & 0xffff;
    // (more than 16 dependencies: the rest polled first, 16 a round; rare)
    for (uint32_t b = 16;; b += 16) {
        const bool more = act && b < depCnt;
        if (!__any(more)) break;
        const uint32_t dd = more && b + t < depCnt ? k.deps[depOff + b + t] : ~0u;
        flow_wait_lanes(dd, k.done, epoch, ctl);
    }
    const uint32_t dep = act && (uint32_t)t < depCnt ? k.deps[depOff + t] : ~0u;
    const int aLim = (int)bits(d[1], 24, 4), lLim = (int)bits(d[1], 28, 4);
    const int na = hA ? (aLim >> 2) + 1 : 0, nl = hL ? (lLim >> 2) + 1 : 0;
    const int nu = na + nl + (hA && hL ? 1 : 0);
    const bool uact = act && t < nu;
    const int kind = t < na ? 0 : t < na + nl ? 1 : 2;  // above, left, corner
    const int u = kind == 0 ? t : t - na;
    const uint32_t masks = bits(d[3], 0, 8), mC = bits(d[3], 8, 2);
    const bool inl = uact && (kind == 0 ? ((masks >> u) & 1) : kind == 1 ? ((masks >> (4 + u)) & 1) : (mC & 1));
    const uint64_t* g = kind == 0 ? gh + (size_t)((y - 1) >> 2) * gw + (x >> 2) + u
                      : kind == 1 ? gv + (size_t)((x - 1) >> 2) * ghn + (y >> 2) + u
                      : (mC & 2) ? gv + (size_t)((x - 1) >> 2) * ghn + ((y - 1) >> 2)
                                 : gh + (size_t)((y - 1) >> 2) * gw + ((x - 1) >> 2);
    uint32_t val = 0;
    // (flow read site: units written in the launch arrive as granules (inl); the frame is read
    // only for pixels final before the launch)
    if (uact && !inl) {
        if (kind == 0) {
            val = ldp4<true>(dst, x + 4 * u, y - 1);
        } else if (kind == 1) {
            const int py = y + 4 * u;
            val = ldp<true>(dst, x - 1, py) | (ldp<true>(dst, x - 1, py + 1) << 8) | (ldp<true>(dst, x - 1, py + 2) << 16) |
                  ((uint32_t)ldp<true>(dst, x - 1, py + 3) << 24);
        } else {
            val = (uint32_t)ldp<true>(dst, x - 1, y - 1) << 24;
        }
    }
    {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t spins = 0, lim = 0;
        bool dead = false, depOk = dep == ~0u, unitOk = !inl;
        for (;;) {
            if (!depOk && !dead) depOk = __hip_atomic_load(k.done + dep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
            if (!unitOk && !dead) {
                const uint64_t v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                unitOk = (uint32_t)(v >> 32) == epoch;
                val = (uint32_t)v;
            }
            if (__all(depOk && unitOk) || dead) break;
            const bool other =
                (spins & AV1R_ERR_POLL_MASK) == 0 && __hip_atomic_load(ctl + FLOW_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            if (!lim) lim = flow_spin_limit(ctl);
            if (other || ++spins > lim || __builtin_amdgcn_s_memrealtime() - t0 > FLOW_WALL) {
                if (lane == 0 && !other) {  // 2: an edge granule wait (as gran_gather)
                    __hip_atomic_store(ctl + FLOW_ERR, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(reinterpret_cast<uint32_t*>(*reinterpret_cast<uint32_t* const*>(ctl + FLOW_HOSTERR)), 2u,
                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                dead = true;
            }
            if (AV1R_POLL_BACKOFF && spins > AV1R_POLL_BACKOFF) __builtin_amdgcn_s_sleep(4);
            else __builtin_amdgcn_s_sleep(1);
        }
    }
    asm volatile("" ::: "memory");  // no pixel load moves above the poll
    TINY_STAMP(4);
    TinyLds& L = T[row];
    if (uact) (kind == 0 ? L.ua + u : kind == 1 ? L.ul + u : L.ul + 7)[0] = val;
    // CFL: the co-located luma of this lane's quad (flow read site: the block's luma, written by
    // the items the dependency list names -- sc1 loads after the wait)
    int cv[4] = {0, 0, 0, 0};
    int csum = 0;
    if (act && cfl && t < nq) {
        const DevPlane luma = P0;
        const int maxLW = (int)(d[3] >> 16), maxLH = (int)(d[4] & 0xffff);
        const int ly = imin((y + qi) << 1, maxLH - 2);
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int lx = imin((x + qj + b) << 1, maxLW - 2);
            const int v = ldp<true>(luma, lx, ly) + ldp<true>(luma, lx + 1, ly) + ldp<true>(luma, lx, ly + 1) + ldp<true>(luma, lx + 1, ly + 1);
            cv[b] = v << 1;
            csum += cv[b];
        }
    }
    coop_sync<64>();  // (wave level: the units are in LDS)
    TINY_STAMP(8);
    // ---- AboveRow / LeftCol (fi_run's passes, per row)
    const uint8_t* ta = reinterpret_cast<const uint8_t*>(L.ua);
    const uint8_t* tl = reinterpret_cast<const uint8_t*>(L.ul);
    const uint8_t* bA = hA ? ta : tl;  // (!hA: the left neighbour (x - 1, y) stands in)
    const uint8_t* bL = hL ? tl : ta;
    const int cA = hA ? aLim : 0, cL = hL ? lLim : 0;
    const bool none = !hA && !hL;
    auto rawA = [&](int i) -> int { const int v = bA[imin(cA, i)]; return none ? 127 : v; };
    auto rawL = [&](int i) -> int { const int v = bL[imin(cL, i)]; return none ? 129 : v; };
    const int c0 = hA && hL ? tl[31] : hA ? ta[0] : tl[0];
    const int corner0 = none ? 128 : c0;
    const int cs = (fl & TI_CORNER) ? r2(rawL(0) * 5 + corner0 * 6 + rawA(0) * 5, 4) : corner0;
    const int strA = (int)bits(d[1], 16, 4), strL = (int)bits(d[1], 20, 4);
    const int nA = (int)bits(d[2], 0, 8), nL = (int)bits(d[2], 8, 8), nUA = (int)bits(d[2], 16, 8), nUL = (int)bits(d[2], 24, 8);
    uint8_t* EA = L.above + TE_OFF;
    uint8_t* EL = L.left + TE_OFF;
    const bool dirc = act && (cls == FI_Z1 || cls == FI_Z2 || cls == FI_Z3);
    const uint8_t* A = EA;
    const uint8_t* Lc = EL;
    const bool filt = (strA | strL) != 0;
    if (__any(dirc)) {
        uint8_t* eA = filt ? L.upA : EA - 1;
        uint8_t* eL = filt ? L.upL : EL - 1;
        if (dirc)
            for (int i = t; i <= w + h; i += 16) {
                eA[i] = (uint8_t)(i == 0 ? cs : rawA(i - 1));
                eL[i] = (uint8_t)(i == 0 ? cs : rawL(i - 1));
            }
        if (__any(dirc && filt)) {
            coop_sync<64>();
            if (dirc && filt)
                for (int i = t; i <= w + h; i += 16) {
                    int a = eA[i], l = eL[i];
                    if (strA && i >= 1 && i < nA) {
                        const int n1 = nA - 1, k0 = fi_ek0(strA), k1 = fi_ek1(strA), k2 = fi_ek2(strA);
                        a = (k0 * (eA[imax(i - 2, 0)] + eA[imin(i + 2, n1)]) + k1 * (eA[i - 1] + eA[imin(i + 1, n1)]) + k2 * a + 8) >> 4;
                    }
                    if (strL && i >= 1 && i < nL) {
                        const int n1 = nL - 1, k0 = fi_ek0(strL), k1 = fi_ek1(strL), k2 = fi_ek2(strL);
                        l = (k0 * (eL[imax(i - 2, 0)] + eL[imin(i + 2, n1)]) + k1 * (eL[i - 1] + eL[imin(i + 1, n1)]) + k2 * l + 8) >> 4;
                    }
                    EA[i - 1] = (uint8_t)a;
                    EL[i - 1] = (uint8_t)l;
                }
        }
        coop_sync<64>();
        // upsampling: buf[2i - 1], buf[2i] from the edge (index -2 .. 2n - 2)
        if (__any(dirc && (nUA | nUL))) {
#pragma unroll
            for (int side = 0; side < 2; side++) {
                const int n = side ? nUL : nUA;
                if (dirc && n) {
                    const uint8_t* e = side ? EL : EA;
                    uint8_t* buf = (side ? L.upL : L.upA) + TE_OFF;
                    if (t < n) {
                        const int d0 = t == 0 ? e[-1] : e[t - 2];
                        const int d1 = e[t - 1], d2 = e[t];
                        const int d3 = t + 1 <= n - 1 ? e[t + 1] : e[n - 1];
                        buf[2 * t - 1] = (uint8_t)clip1(r2(-d0 + 9 * d1 + 9 * d2 - d3, 4));
                        buf[2 * t] = (uint8_t)d2;
                    }
                    if (t == 0) buf[-2] = e[-1];
                }
            }
            coop_sync<64>();
            if (nUA) A = L.upA + TE_OFF;
            if (nUL) Lc = L.upL + TE_OFF;
        }
    }
    // DC (and CFL's DC): the edge sums over the row
    int dc = 128;
    {
        const int v = act && cls == FI_DC ? (hA && t < w ? rawA(t) : 0) + (hL && t < h ? rawL(t) : 0) : 0;
        const int s = row16_total(v);
        if (hA && hL) {
            // (s + (w + h) / 2) / (w + h): a shift when square, else w + h = 12 (4x8, 8x4):
            // the quotient from a float reciprocal corrected by one either way (as fi_run)
            const int n = s + ((w + h) >> 1);
            if (log2W == log2H) {
                dc = n >> (log2W + 1);
            } else {
                const int dd = w + h;
                int q = (int)((float)n * __builtin_amdgcn_rcpf((float)dd));
                q += (q + 1) * dd <= n;
                q -= q * dd > n;
                dc = q;
            }
        } else if (hL) {
            dc = clip1((s + (h >> 1)) >> log2H);
        } else if (hA) {
            dc = clip1((s + (w >> 1)) >> log2W);
        }
    }
    // ---- this lane's quad
    uint32_t p = 0;
    if (act && t < nq) {
        const int i = qi;
        const int upA = nUA ? 1 : 0, upL = nUL ? 1 : 0;
        const int dx = (int)(d[3] >> 16), dy = (int)(d[4] & 0xffff);
        switch (cls) {
        case FI_DC: p = (uint32_t)dc * 0x01010101u; break;
        case FI_V: p = rawA(qj) | rawA(qj + 1) << 8 | rawA(qj + 2) << 16 | (uint32_t)rawA(qj + 3) << 24; break;
        case FI_H: p = (uint32_t)rawL(i) * 0x01010101u; break;
        case FI_Z1: {
            const int idx = (i + 1) * dx;
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
                int idx = (j << 6) - (i + 1) * dx;
                int base = idx >> (6 - upA);
                int v;
                if (base >= -(1 << upA)) {
                    const int shift = ((idx << upA) >> 1) & 0x1F;
                    v = r2(A[base] * (32 - shift) + A[base + 1] * shift, 5);
                } else {
                    idx = (i << 6) - (j + 1) * dy;
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
                const int idx = (qj + b + 1) * dy;
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
                if (cls == FI_SMOOTH) v = r2(wy * a + (256 - wy) * bl + wx * l + (256 - wx) * tr, 9);
                else if (cls == FI_SMOOTH_V) v = r2(wy * a + (256 - wy) * bl, 8);
                else v = r2(wx * l + (256 - wx) * tr, 8);
                p |= (uint32_t)v << (8 * b);
            }
            break;
        }
        }
    }
    {
        // CFL: the luma average over the block (every quad of a tiny item is in its row)
        const int s = row16_total(csum);
        if (act && cfl) {
            const int alpha = (int)(int8_t)bits(d[4], 16, 8);
            const int avg = r2(s, log2W + log2H);
            uint32_t q = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) q |= (uint32_t)clip1(dc + r2s(alpha * (cv[b] - avg), 6)) << (8 * b);
            p = q;
        }
    }
    const uint32_t o = add4(p, res);
    TINY_STAMP(9);
    // ---- the granules first (what the next items wait for), then the frame (as fi_run: the
    // bottom row's units are the last row's quads; a right-column unit is byte 3 of four
    // vertically adjacent quads, t + w4, + 2 w4, + 3 w4 -- in the same DPP row)
    const uint64_t tag = (uint64_t)epoch << 32;
    const uint32_t a1 = __builtin_amdgcn_update_dpp(0, (int)o, 0x101, 0xf, 0xf, true);  // row_shl:1
    const uint32_t a2 = __builtin_amdgcn_update_dpp(0, (int)o, 0x102, 0xf, 0xf, true);
    const uint32_t a3 = __builtin_amdgcn_update_dpp(0, (int)o, 0x103, 0xf, 0xf, true);
    const uint32_t b2 = __builtin_amdgcn_update_dpp(0, (int)o, 0x104, 0xf, 0xf, true);
    const uint32_t b3 = __builtin_amdgcn_update_dpp(0, (int)o, 0x106, 0xf, 0xf, true);
    const uint32_t o1 = w4 == 1 ? a1 : a2, o2 = w4 == 1 ? a2 : b2, o3 = w4 == 1 ? a3 : b3;
    if (act && t < nq && qi == h - 1)
        __hip_atomic_store(const_cast<uint64_t*>(gh) + (size_t)((y + h - 1) >> 2) * gw + (x >> 2) + (qj >> 2), tag | o,
            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (act && t < nq && qj == w - 4 && (qi & 3) == 0) {
        const uint32_t v = (o >> 24) | ((o1 >> 24) << 8) | ((o2 >> 24) << 16) | ((o3 >> 24) << 24);
        __hip_atomic_store(const_cast<uint64_t*>(gv) + (size_t)((x + w - 1) >> 2) * ghn + (y >> 2) + (qi >> 2), tag | v,
            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (act && t < nq) stp4<true>(dst, x + qj, y + qi, o);
    TINY_STAMP(10);
    // the drain and done flag where a dependency list names the item (CFL's luma)
    const bool pub = act && (fl & TI_PUB);
    if (__any(pub)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (pub && t == 0) __hip_atomic_store(k.done + pos, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    TINY_STAMP(5);
}

// groups[g] = {frame << 8 | n, first item position}: n = 0 one large item (the whole
// workgroup), n | FLOW_G_TINY: n tiny items (four per wave, tiny_run), else n >= 1 small
// items (wave w runs items w, w + 4, ..)
#ifndef AV1R_FLOW_WAVES
#define AV1R_FLOW_WAVES 6  // resident 256-lane workgroups per CU: 6 = 80 VGPRs (round 6, with the tiny path: k_flow -2.4 %, profiles/r06_ab_flow_waves6.txt); 5 = 95 VGPRs; 4 = 121 VGPRs: +2.4 %; 8 = 64 VGPRs + spills: 4K recon +3 %, profiles/r05_ab_flow_waves8.txt
#endif
#ifdef AV1R_FLOW_DEBUG
// -DAV1R_FLOW_DEBUG: counts workgroup entries that find another launch's k_flow
// workgroups still running (co-resident grids, which the flow chain should exclude), and
// records the first FLOW_DBG_PAIRS (earlier epoch, entering epoch) pairs.  g_flow_active
// holds, per epoch slot (epoch % 64), that launch's running workgroups, so an entry is an
// overlap exactly when another slot is non-zero (one atomic per slot, no cross-word race).
#define FLOW_DBG_PAIRS 256
__device__ uint32_t g_flow_active[64], g_flow_overlap, g_flow_pairs[FLOW_DBG_PAIRS];
#endif
extern "C" __global__ __launch_bounds__(256, AV1R_FLOW_WAVES) void k_flow(const KParams* kps, const uint2* __restrict__ groups, uint32_t nGroups,
    uint32_t* ctl, uint32_t epoch, unsigned long long* trace)
{
    constexpr size_t kLds = sizeof(TbLds<64>) > 4 * sizeof(TbLds<TB_SMALL>) ? sizeof(TbLds<64>) : 4 * sizeof(TbLds<TB_SMALL>);
    static_assert(16 * sizeof(TinyLds) <= kLds, "k_flow LDS: the tiny groups' rows");
    __shared__ __align__(16) uint8_t smem[kLds];
    __shared__ uint32_t ticket[2];  // double-buffered: a slow wave may still read the old one
    // The queue a workgroup serves is its ENTRY order, not its blockIdx: the first
    // FLOW_QUEUES workgroups to start cover every queue wherever the dispatcher put them.
    // (blockIdx % 8 is also the XCD a workgroup lands on: with queue = blockIdx % 8 every
    // queue lived on one XCD, and two overlapping grids could each fill an XCD the other
    // needed -- grid A's queue-q groups waiting for a slot on XCD q held by grid B's spinning
    // workgroups, and B's the other way round: the cross-stream timeout of round 1.)
    __shared__ uint32_t qsh;
    if (threadIdx.x == 0) {
        const uint32_t e = __hip_atomic_fetch_add(ctl + FLOW_ASSIGN, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        qsh = e % FLOW_QUEUES;
#ifdef AV1R_FLOW_DEBUG
        atomicAdd(&g_flow_active[epoch & 63], 1u);
        for (uint32_t e = 1; e < 64; e++) {
            const uint32_t o = (epoch + e) & 63;
            if (__hip_atomic_load(&g_flow_active[o], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                const uint32_t k = atomicAdd(&g_flow_overlap, 1u);
                if (k < FLOW_DBG_PAIRS) g_flow_pairs[k] = (o << 16) | (epoch & 0xffff);
                break;
            }
        }
#endif
    }
    __syncthreads();
    const uint32_t q = __builtin_amdgcn_readfirstlane(qsh);
    uint32_t* head = ctl + q * FLOW_LINE;
    if (threadIdx.x == 0) ticket[0] = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    for (uint32_t it = 0;; it ^= 1) {
        const uint32_t g = __builtin_amdgcn_readfirstlane(ticket[it]) * FLOW_QUEUES + q;
        if (g >= nGroups) {
#ifdef AV1R_FLOW_DEBUG
            if (threadIdx.x == 0) atomicSub(&g_flow_active[epoch & 63], 1u);
#endif
            return;
        }
        // (the next ticket is taken after the group: taken before it, its round trip hidden
        // behind the group's work, k_flow measured 0.060 -> 0.070 ms/frame in round 5 -- a held
        // ticket delays the group most likely on the critical path)
        const uint2 gd = groups[g];
        const KParams& k = KP(kps, gd.x >> 8);
        const uint32_t n = gd.x & 0xff;
        if (n == 0) {
            flow_item<256, 64>(k, gd.y, *reinterpret_cast<TbLds<64>*>(smem), epoch, ctl, trace, gd.x >> 8);
        } else if (n & FLOW_G_TINY) {
            // tiny items: wave w runs items w, w + 4, w + 8, w + 12 side by side (tiny_run)
            const uint32_t nt = n & (FLOW_G_TINY - 1);
            const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            if (wave < nt) tiny_run(k, gd.y, nt, reinterpret_cast<TinyLds*>(smem) + 4 * wave, epoch, ctl, trace, gd.x >> 8);
        } else {
            // small items: wave w runs items w, w + 4, .. of the group, one after the other in
            // its own LDS tiles (the host's groups hold 4, or 8 on crowded levels: items of
            // one level, none waiting for another)
            const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (a scalar branch: no item code runs with exec = 0)
            for (uint32_t w = wave; w < n; w += 4)
                flow_item<64, TB_SMALL>(k, gd.y + w, reinterpret_cast<TbLds<TB_SMALL>*>(smem)[wave], epoch, ctl, trace,
                    gd.x >> 8);
        }
        if (threadIdx.x == 0) ticket[it ^ 1] = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();  // the LDS tiles are free again; the next ticket is published
    }
}

// persistent grid of k_flow on `device`: every CU's resident workgroups (capped at 8 per
// CU), a multiple of FLOW_QUEUES
int flow_grid(int device, int maxPer)
{
    static int cache[64][9] = {};  // per device and workgroups-per-CU bound (1..8)
    if (device < 0 || device >= 64) return FLOW_QUEUES;
    const int slot = maxPer < 1 ? 1 : (maxPer > 8 ? 8 : maxPer);
    if (!cache[device][slot]) {
        int cus = 0, per = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 32;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(k_flow), 256, 0) != hipSuccess || per <= 0)
            per = 1;
        per = per > 8 ? 8 : per;
        per = per > maxPer ? maxPer : per;
        int g = ((cus * per) / FLOW_QUEUES) * FLOW_QUEUES;
        cache[device][slot] = g < FLOW_QUEUES ? FLOW_QUEUES : g;
    }
    return cache[device][slot];
}

#ifdef AV1R_FLOW_DEBUG
// overlap count since the last reset; pairs[] (up to n) the (earlier epoch slot << 16 |
// entering epoch) of the first overlaps; reset = 1 zeroes the counters afterwards
uint32_t flow_debug_overlaps(uint32_t* pairs, int n, int reset)
{
    uint32_t v = 0;
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_flow_overlap), sizeof(v));
    if (pairs && n > 0) (void)hipMemcpyFromSymbol(pairs, HIP_SYMBOL(g_flow_pairs), 4 * (n < FLOW_DBG_PAIRS ? n : FLOW_DBG_PAIRS));
    if (reset) {
        const uint32_t z[64] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_flow_overlap), z, 4);
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_flow_active), z, sizeof(z));
        (void)hipDeviceSynchronize();
    }
    return v;
}
#endif

void launch_k_flow(const KParams* kps, const void* groups, uint32_t nGroups, uint32_t* ctl, uint32_t* hostErr,
    uint32_t epoch, int grid, unsigned long long* trace, hipStream_t s)
{
    (void)hostErr;  // (its address travels in the control block: FLOW_HOSTERR)
    hipLaunchKernelGGL(k_flow, dim3(grid), dim3(256), 0, s, kps, reinterpret_cast<const uint2*>(groups), nGroups, ctl, epoch,
        trace);
}

#endif  // AV1R_FLOW_PART

#ifndef AV1R_FLOW_PART
// ---------------------------------------------------------------------------------
// k_resid (k_flow mode, after k_inter): the residual of every TB with coefficients
// (TransformBlock::reconstruct + inverseTransform, TransformBlock.cpp:2173-2276), with no
// dependencies at all.  An inter TB outside an inter-intra block is added to its
// prediction in the frame right here (TransformBlock.cpp:2440-2456); every other residual
// is stored as an int16 tile for the k_flow item (intra TB, inter-intra blend) that adds
// it.  k_resid_s: 64 4x4 TBs (4 lanes each) or 16 other TBs with sides <= 16 (16 lanes
// each) per 256-lane workgroup;
// k_resid_l: one larger TB per 64-lane workgroup.  tab: [prefix of the frames' workgroup
// counts (n + 1)].
// ---------------------------------------------------------------------------------
template <int NT, int MAX>
DEV void resid_one(const KParams& k, uint32_t ti, int16_t* res)
{
    constexpr int RS = MAX + 2;
    const int t = coop_lane<NT>();
    const DevTb& tb = k.tbs[ti];
    const uint32_t c0 = t < tb.coef_cnt ? coef_at(k, tb.coef_off, tb.flags, t) : 0u;
    const DevBlock& blk = k.blocks[tb.block];
    const uint32_t ro = k.tb_res[ti];
    tb_residual<NT, MAX>(k, tb, blk, res, c0);
    const int l2q = av1r_tx_w_log2[tb.tx_size] - 2;
    const int nq = (av1r_tx_w[tb.tx_size] * av1r_tx_h[tb.tx_size]) >> 2;
    const DevPlane& dst = k.cur.pl[tb.plane];
    for (int q = t; q < nq; q += NT) {
        const int i = q >> l2q, j = (q & ((1 << l2q) - 1)) << 2;
        const uint32_t r01 = *reinterpret_cast<const uint32_t*>(&res[i * RS + j]);
        const uint32_t r23 = *reinterpret_cast<const uint32_t*>(&res[i * RS + j + 2]);
        if (ro == ~0u) stp4<false>(dst, tb.x + j, tb.y + i, add4(ldp4<false>(dst, tb.x + j, tb.y + i), make_uint2(r01, r23)));
        else reinterpret_cast<uint2*>(k.res + ro)[q] = make_uint2(r01, r23);
    }
}

// (a frame's first n_resid_t workgroups take 64 4x4 TBs at 4 lanes each: with 16 lanes a
// 4x4 TB -- half the TBs with coefficients -- left 12 idle through both passes; the next
// n_resid_e 32 TBs of at most 8x8 at 8 lanes each, round 6)
extern "C" __global__ __launch_bounds__(256) void k_resid_s(const KParams* kps, const uint32_t* __restrict__ tab, int n)
{
    __shared__ __align__(16) union {
        int16_t s[16][16 * 18];
        int16_t e[32][8 * 10];
        int16_t t[64][4 * 6];
    } res;
    const uint32_t b = xcd_order(blockIdx.x, gridDim.x);
    const int lane = threadIdx.x & 63;
    const uint32_t pre = lane + 1 < n ? tab[lane + 1] : 0xffffffffu;
    const int s = __builtin_amdgcn_readfirstlane(__popcll(__ballot(b >= pre)));
    const KParams& k = KP(kps, s);
    const uint32_t bl = b - tab[s], nt = k.n_resid_t, ne = k.n_resid_e;
    if (bl < nt) {
        const int g = threadIdx.x >> 2;
        const uint32_t ti = k.resid_s[bl * 64 + g];
        if (ti != ~0u) resid_one<4, 4>(k, ti, res.t[g]);
        return;
    }
    if (bl < nt + ne) {  // 32 TBs of at most 8x8 (8x8, 8x4, 4x8), 8 lanes each
        const int g = threadIdx.x >> 3;
        const uint32_t ti = k.resid_s[nt * 64 + (bl - nt) * 32 + g];
        if (ti != ~0u) resid_one<8, 8>(k, ti, res.e[g]);
        return;
    }
    const int g = threadIdx.x >> 4;
    const uint32_t ti = k.resid_s[nt * 64 + ne * 32 + (bl - nt - ne) * 16 + g];
    if (ti != ~0u) resid_one<16, 16>(k, ti, res.s[g]);
}

extern "C" __global__ __launch_bounds__(64) void k_resid_l(const KParams* kps, const uint32_t* __restrict__ tab, int n)
{
    __shared__ __align__(16) union {
        int16_t l[64 * 66];
        int16_t m[2][32 * 34];
    } res;
    const uint32_t b = xcd_order(blockIdx.x, gridDim.x);
    const int lane = threadIdx.x & 63;
    const uint32_t pre = lane + 1 < n ? tab[lane + 1] : 0xffffffffu;
    const int s = __builtin_amdgcn_readfirstlane(__popcll(__ballot(b >= pre)));
    const KParams& k = KP(kps, s);
    const uint32_t bl = b - tab[s], nm = sload(k.resid_l);  // (the list's head: its pair count)
    if (bl < nm) {  // two TBs of at most 32x32, 32 lanes each (round 6)
        const int g = lane >> 5;
        const uint32_t ti = k.resid_l[1 + 2 * bl + g];
        if (ti != ~0u) resid_one<32, 32>(k, ti, res.m[g]);
        return;
    }
    resid_one<64, 64>(k, k.resid_l[1 + 2 * nm + (bl - nm)], res.l);
}

void launch_k_resid(int large, const KParams* kps, const uint32_t* tab, int n, unsigned groups, hipStream_t s)
{
    if (large) hipLaunchKernelGGL(k_resid_l, dim3(groups), dim3(64), 0, s, kps, tab, n);
    else hipLaunchKernelGGL(k_resid_s, dim3(groups), dim3(256), 0, s, kps, tab, n);
}

// kind 0: inter tiles, `items` workgroups; kind 1: `items` = big items + ceil(small / 4);
// kind 2 / 3: medium / small plain inter blocks, `items` groups of two / four
void launch_k_inter_all(const KParams* kps, const uint32_t* tab, int n, uint32_t gI, uint32_t gM, uint32_t gS, uint32_t nb,
    unsigned long long* trace, hipStream_t s)
{
    hipLaunchKernelGGL(k_inter_all, dim3(gI + gM + gS), dim3(64), 0, s, kps, tab, n, gI, gM, gS, nb, trace);
}
void launch_k_level(int kind, const KParams* kps, const uint32_t* tab, int n, unsigned items, unsigned long long* trace,
    uint32_t traceBase, hipStream_t s)
{
    if (kind == 0) hipLaunchKernelGGL(k_inter, dim3(items), dim3(64), 0, s, kps, tab, n, trace, traceBase);
    else if (kind == 2) hipLaunchKernelGGL(k_inter_m, dim3(items), dim3(64), 0, s, kps, tab, n);
    else if (kind == 3) hipLaunchKernelGGL(k_inter_s, dim3(items), dim3(64), 0, s, kps, tab, n);
    else hipLaunchKernelGGL(k_tb, dim3(items), dim3(256), 0, s, kps, tab, n, trace, traceBase);
}
#endif  // !AV1R_FLOW_PART
