/*
 * av1r_oracle.c -- CPU restatement of the reference decoder's reconstruction and
 * in-loop filter path (oddstone/av1dec), consuming the av1r frame batch (include/av1r.h).
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker for the HIP backend and the
 * "port" CPU baseline in bench.py.  Nothing in the product (av1dec_amd/) links, loads or
 * calls it.  It is pinned against the reference itself: tests/test_oracle.py replays the
 * batches that oracle/harness/refdump.cpp extracted from the reference for all 172
 * conformance streams and requires every per-stage MD5 (recon / LF / CDEF / LR) and the
 * whole-output MD5 of bits/bits.md5 to match.
 *
 * It follows the reference statement by statement, single-threaded, including the
 * reference's frame-buffer geometry (YuvFrame, decoder/VideoFrame.cpp:38-101) so that
 * pixels outside the visible area evolve exactly as in the reference.  Every function
 * cites the reference code it restates.
 */
#include "av1r.h"
#include "av1r_consts.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define CLIP3(lo, hi, v) ((v) < (lo) ? (lo) : ((v) > (hi) ? (hi) : (v)))
#define CLIP1(v) CLIP3(0, 255, (v))
#define MIN(a, b) ((a) < (b) ? (a) : (b))
#define MAX(a, b) ((a) > (b) ? (a) : (b))

/* ROUND2 / ROUND2SIGNED (decoder/Av1Common.h:174-178) */
static inline int r2(int x, int n) { return n == 0 ? x : ((x + (1 << (n - 1))) >> n); }
static inline int r2s(int x, int n) { return x >= 0 ? r2(x, n) : -r2(-x, n); }
static inline int64_t r2_64(int64_t x, int n) { return n == 0 ? x : ((x + ((int64_t)1 << (n - 1))) >> n); }
static inline int64_t r2s_64(int64_t x, int n) { return x >= 0 ? r2_64(x, n) : -r2_64(-x, n); }
static inline int iabs(int v) { return v < 0 ? -v : v; }
static int floor_log2(int64_t x) { int s = 0; while (x) { x >>= 1; s++; } return s - 1; }

/* ------------------------------------------------------------------------------------
 * Frame buffers: YuvFrame::create (VideoFrame.cpp:38-62), copy-create (:64-79),
 * extendBorder (:81-101).  Refcounted because the reference shares frames between the
 * output FIFO and the FrameStore (Av1Decoder.cpp:111-119, 150-153).
 * ---------------------------------------------------------------------------------- */
typedef struct OFrame {
    int refcnt;
    int width, height;
    uint8_t* mem;
    uint8_t* data[3];
    int stride[3], w[3], h[3];
} OFrame;

#define PAD 16
static OFrame* frame_create(int width, int height)
{
    OFrame* f = (OFrame*)calloc(1, sizeof(OFrame));
    int aw = (width + 127) & ~127, ah = (height + 127) & ~127;
    int allocW = aw + PAD * 2, allocH = ah + PAD * 2;
    f->mem = (uint8_t*)calloc((size_t)allocW * allocH * 3 / 2, 1);
    f->refcnt = 1;
    f->width = width;
    f->height = height;
    static const int sub[3] = {1, 2, 2};
    const double off[3] = {0, 1, 5.0 / 4};
    for (int i = 0; i < 3; i++) {
        f->w[i] = width / sub[i];
        f->h[i] = height / sub[i];
        f->stride[i] = allocW / sub[i];
        f->data[i] = f->mem + (int)(allocW * allocH * off[i]) + (PAD * f->stride[i] + PAD) / sub[i];
    }
    return f;
}
static OFrame* frame_copy(const OFrame* o)
{
    OFrame* f = frame_create(o->width, o->height);
    for (int p = 0; p < 3; p++)
        for (int y = 0; y < o->h[p]; y++)
            memcpy(f->data[p] + y * f->stride[p], o->data[p] + y * o->stride[p], o->w[p]);
    return f;
}
static void frame_ref(OFrame* f) { if (f) f->refcnt++; }
static void frame_unref(OFrame* f)
{
    if (f && --f->refcnt == 0) {
        free(f->mem);
        free(f);
    }
}
static void frame_extend_border(OFrame* f, int borders)
{
    for (int p = 0; p < 3; p++) {
        uint8_t* dest = f->data[p];
        int s = f->stride[p];
        for (int y = 0; y < f->h[p]; y++) {
            uint8_t* d = dest + y * s;
            memset(d - borders, d[0], borders);
            d += f->w[p];
            memset(d, d[-1], borders);
        }
        uint8_t* top = dest - borders;
        uint8_t* bottom = top + (f->h[p] - 1) * s;
        int size = f->w[p] + 2 * borders;
        for (int i = 1; i <= borders; i++) {
            memcpy(top - i * s, top, size);
            memcpy(bottom + i * s, bottom, size);
        }
    }
}
#define PIX(f, p, x, y) ((f)->data[p][(y) * (f)->stride[p] + (x)])

/* ------------------------------------------------------------------------------------ */
typedef struct oracle_ctx {
    OFrame* store[8];
    OFrame** outq;
    int nout, capout, headout;
    OFrame* stage[4];
    int keep_stages;
    /* current frame */
    const av1r_frame_batch* b;
    const av1r_frame_hdr* h;
    OFrame* cur;
    /* compute_prediction's shared mask (Block.cpp:104) and InterPredict::preds */
    uint8_t mask[128][128];
    int16_t preds[2][128][128];
} oracle_ctx;

static const av1r_mi* mi_at(const oracle_ctx* c, int row, int col)
{
    return &c->b->mi[(size_t)row * c->h->mi_stride + col];
}
static int plane_size(int bs, int plane) { return plane ? av1r_ss420[bs] : bs; }

/* ======================================================================================
 * Intra prediction (decoder/IntraPredict.cpp)
 * ==================================================================================== */
typedef struct IntraArgs {
    int plane, x, y, log2W, log2H;
    const av1r_block* blk;
} IntraArgs;

/* recursiveIntraPrediction (IntraPredict.cpp:112-149) */
static void filter_intra(const IntraArgs* a, const uint8_t* above, const uint8_t* left, uint8_t* pred)
{
    int w = 1 << a->log2W, h = 1 << a->log2H;
    int w4 = w >> 2, h2 = h >> 1;
    int mode = a->blk->filter_intra_mode;
    for (int i2 = 0; i2 < h2; i2++) {
        for (int j4 = 0; j4 < w4; j4++) {
            int p[7];
            for (int i = 0; i < 5; i++) {
                if (!i2)
                    p[i] = above[(j4 << 2) + i - 1];
                else if (!j4 && !i)
                    p[i] = left[(i2 << 1) - 1];
                else
                    p[i] = pred[((i2 << 1) - 1) * 64 + (j4 << 2) + i - 1];
            }
            for (int i = 5; i < 7; i++) {
                if (!j4)
                    p[i] = left[(i2 << 1) + i - 5];
                else
                    p[i] = pred[((i2 << 1) + i - 5) * 64 + (j4 << 2) - 1];
            }
            for (int i1 = 0; i1 < 2; i1++) {
                for (int j1 = 0; j1 < 4; j1++) {
                    int pr = 0;
                    for (int i = 0; i < 7; i++)
                        pr += av1r_filter_intra_taps[(mode * 8 + (i1 << 2) + j1) * 7 + i] * p[i];
                    pred[((i2 << 1) + i1) * 64 + (j4 << 2) + j1] = (uint8_t)CLIP1(r2s(pr, 4));
                }
            }
        }
    }
}

static int get_dx(int pAngle)
{
    if (pAngle < 90)
        return av1r_dr_intra_derivative[pAngle];
    if (pAngle > 90 && pAngle < 180)
        return av1r_dr_intra_derivative[180 - pAngle];
    return 0;
}
static int get_dy(int pAngle)
{
    if (pAngle > 90 && pAngle < 180)
        return av1r_dr_intra_derivative[pAngle - 90];
    if (pAngle > 180)
        return av1r_dr_intra_derivative[270 - pAngle];
    return 0;
}

/* getIntraEdgeFilterStrength (IntraPredict.cpp:256-306) */
static int edge_strength(int w, int h, int filterType, int delta)
{
    int d = iabs(delta), blkWh = w + h, s = 0;
    if (!filterType) {
        if (blkWh <= 8) {
            if (d >= 56) s = 1;
        } else if (blkWh <= 12) {
            if (d >= 40) s = 1;
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
/* intraEdgeFilter (IntraPredict.cpp:324-337) */
static void edge_filter(int sz, int strength, uint8_t* array)
{
    if (!strength)
        return;
    uint8_t edge[300];
    memcpy(edge, array - 1, sz);
    for (int i = 1; i < sz; i++) {
        int s = 0;
        for (int j = 0; j < 5; j++) {
            int k = CLIP3(0, sz - 1, i - 2 + j);
            s += av1r_edge_kernel[strength - 1][j] * edge[k];
        }
        array[i - 1] = (uint8_t)((s + 8) >> 4);
    }
}
/* getIntraEdgeUpsample (IntraPredict.cpp:339-352) */
static int edge_upsample_used(int w, int h, int filterType, int delta)
{
    int d = iabs(delta), blkWh = w + h;
    if (d <= 0 || d >= 40)
        return 0;
    return filterType ? (blkWh <= 8) : (blkWh <= 16);
}
/* intraEdgeUpsample (IntraPredict.cpp:354-370); returns pointer to buf[0] inside `up` */
static uint8_t* edge_upsample(const uint8_t* edge, int numPx, uint8_t* up)
{
    uint8_t dup[80];
    dup[0] = edge[-1];
    for (int i = -1; i < numPx; i++)
        dup[i + 2] = edge[i];
    dup[numPx + 2] = edge[numPx - 1];
    uint8_t* buf = up + 2;
    buf[-2] = dup[0];
    for (int i = 0; i < numPx; i++) {
        int s = -dup[i] + 9 * dup[i + 1] + 9 * dup[i + 2] - dup[i + 3];
        buf[2 * i - 1] = (uint8_t)CLIP1(r2(s, 4));
        buf[2 * i] = dup[i + 2];
    }
    return buf;
}

/* directionalIntraPredict (IntraPredict.cpp:379-483) */
static void directional(const oracle_ctx* c, const IntraArgs* a, int haveAbove, int haveLeft,
    uint8_t* above, uint8_t* left, int mode, uint8_t* pred)
{
    const av1r_frame_hdr* h = c->h;
    int plane = a->plane, x = a->x, y = a->y;
    int w = 1 << a->log2W, hh = 1 << a->log2H;
    int subX = plane ? h->subx : 0, subY = plane ? h->suby : 0;
    int maxX = (h->mi_cols * 4) >> subX;
    int maxY = (h->mi_rows * 4) >> subY;
    int angleDelta = plane == 0 ? a->blk->angle_delta_y : a->blk->angle_delta_uv;
    int pAngle = av1r_mode_to_angle[mode] + angleDelta * 3;
    int upA = 0, upL = 0;
    uint8_t upbufA[300], upbufL[300];
    if (h->enable_intra_edge_filter) {
        if (pAngle != 90 && pAngle != 180) {
            if (pAngle > 90 && pAngle < 180 && (w + hh) >= 24) {
                /* filterCorner (IntraPredict.cpp:204-209) */
                uint8_t s = (uint8_t)r2(left[0] * 5 + above[-1] * 6 + above[0] * 5, 4);
                left[-1] = s;
                above[-1] = s;
            }
            uint32_t f = a->blk->flags;
            int filterType = plane ? ((f & AV1R_BLK_SMOOTH_A_UV) || (f & AV1R_BLK_SMOOTH_L_UV))
                                   : ((f & AV1R_BLK_SMOOTH_A_Y) || (f & AV1R_BLK_SMOOTH_L_Y));
            if (haveAbove) {
                int strength = edge_strength(w, hh, filterType, pAngle - 90);
                int numPx = MIN(w, (maxX - x + 1)) + (pAngle < 90 ? hh : 0) + 1;
                edge_filter(numPx, strength, above);
            }
            if (haveLeft) {
                int strength = edge_strength(w, hh, filterType, pAngle - 180);
                int numPx = MIN(hh, (maxY - y + 1)) + (pAngle > 180 ? w : 0) + 1;
                edge_filter(numPx, strength, left);
            }
            upA = edge_upsample_used(w, hh, filterType, pAngle - 90);
            if (upA)
                above = edge_upsample(above, w + (pAngle < 90 ? hh : 0), upbufA);
            upL = edge_upsample_used(w, hh, filterType, pAngle - 180);
            if (upL)
                left = edge_upsample(left, hh + (pAngle > 180 ? w : 0), upbufL);
        }
    }
    if (pAngle < 90) {
        int dx = get_dx(pAngle);
        int maxBaseX = (w + hh - 1) << upA;
        for (int i = 0; i < hh; i++)
            for (int j = 0; j < w; j++) {
                int idx = (i + 1) * dx;
                int base = (idx >> (6 - upA)) + (j << upA);
                int shift = ((idx << upA) >> 1) & 0x1F;
                pred[i * 64 + j] = base < maxBaseX
                    ? (uint8_t)r2(above[base] * (32 - shift) + above[base + 1] * shift, 5)
                    : above[maxBaseX];
            }
    } else if (pAngle > 90 && pAngle < 180) {
        int dx = get_dx(pAngle), dy = get_dy(pAngle);
        for (int i = 0; i < hh; i++)
            for (int j = 0; j < w; j++) {
                int idx = (j << 6) - (i + 1) * dx;
                int base = idx >> (6 - upA);
                if (base >= -(1 << upA)) {
                    int shift = ((idx << upA) >> 1) & 0x1F;
                    pred[i * 64 + j] = (uint8_t)r2(above[base] * (32 - shift) + above[base + 1] * shift, 5);
                } else {
                    idx = (i << 6) - (j + 1) * dy;
                    base = idx >> (6 - upL);
                    int shift = ((idx << upL) >> 1) & 0x1F;
                    pred[i * 64 + j] = (uint8_t)r2(left[base] * (32 - shift) + left[base + 1] * shift, 5);
                }
            }
    } else if (pAngle > 180) {
        int dy = get_dy(pAngle);
        for (int i = 0; i < hh; i++)
            for (int j = 0; j < w; j++) {
                int idx = (j + 1) * dy;
                int base = (idx >> (6 - upL)) + (i << upL);
                int shift = ((idx << upL) >> 1) & 0x1F;
                pred[i * 64 + j] = (uint8_t)r2(left[base] * (32 - shift) + left[base + 1] * shift, 5);
            }
    } else if (pAngle == 90) {
        for (int i = 0; i < hh; i++)
            for (int j = 0; j < w; j++)
                pred[i * 64 + j] = above[j];
    } else {
        for (int i = 0; i < hh; i++)
            for (int j = 0; j < w; j++)
                pred[i * 64 + j] = left[i];
    }
}

static const uint8_t* sm_weights(int log2) { return av1r_sm_weights + ((1 << log2) - 4); }

/* predict_intra (IntraPredict.cpp:563-630) + the predictors it dispatches to */
static void predict_intra(const oracle_ctx* c, const IntraArgs* a, int haveLeft, int haveAbove,
    int haveAR, int haveBL, int mode, uint8_t* pred)
{
    const av1r_frame_hdr* h = c->h;
    const OFrame* f = c->cur;
    int plane = a->plane, x = a->x, y = a->y;
    int w = 1 << a->log2W, hh = 1 << a->log2H;
    int subX = plane ? h->subx : 0;
    int subY = plane ? h->subx : 0; /* the reference uses subsampling_x here (IntraPredict.cpp:567) */
    int maxX = ((h->mi_cols * 4) >> subX) - 1;
    int maxY = ((h->mi_rows * 4) >> subY) - 1;
    uint8_t aboveRow[300], leftCol[300];
    uint8_t* above = aboveRow + 16;
    uint8_t* left = leftCol + 16;
    const int median = 128;
    if (!haveAbove && haveLeft) {
        uint8_t v = PIX(f, plane, x - 1, y);
        for (int i = 0; i < w + hh; i++) above[i] = v;
    } else if (!haveAbove && !haveLeft) {
        for (int i = 0; i < w + hh; i++) above[i] = median - 1;
    } else {
        int aboveLimit = MIN(maxX, x + (haveAR ? 2 * w : w) - 1);
        for (int i = 0; i < w + hh; i++)
            above[i] = PIX(f, plane, MIN(aboveLimit, x + i), y - 1);
    }
    if (!haveLeft && haveAbove) {
        uint8_t v = PIX(f, plane, x, y - 1);
        for (int i = 0; i < w + hh; i++) left[i] = v;
    } else if (!haveAbove && !haveLeft) {
        for (int i = 0; i < w + hh; i++) left[i] = median + 1;
    } else {
        int leftLimit = MIN(maxY, y + (haveBL ? 2 * hh : hh) - 1);
        for (int i = 0; i < w + hh; i++)
            left[i] = PIX(f, plane, x - 1, MIN(leftLimit, y + i));
    }
    if (haveAbove && haveLeft)
        above[-1] = PIX(f, plane, x - 1, y - 1);
    else if (haveAbove)
        above[-1] = PIX(f, plane, x, y - 1);
    else if (haveLeft)
        above[-1] = PIX(f, plane, x - 1, y);
    else
        above[-1] = median;
    left[-1] = above[-1];

    if (plane == 0 && (a->blk->flags & AV1R_BLK_FILTER_INTRA)) {
        filter_intra(a, above, left, pred);
    } else if (mode >= AV1R_V_PRED && mode <= AV1R_D67_PRED) {
        directional(c, a, haveAbove, haveLeft, above, left, mode, pred);
    } else if (mode == AV1R_PAETH_PRED) {
        /* paethPredict (IntraPredict.cpp:151-171) */
        for (int i = 0; i < hh; i++)
            for (int j = 0; j < w; j++) {
                int base = above[j] + left[i] - above[-1];
                int pL = iabs(base - left[i]), pT = iabs(base - above[j]), pTL = iabs(base - above[-1]);
                pred[i * 64 + j] = (pL <= pT && pL <= pTL) ? left[i] : (pT <= pTL ? above[j] : above[-1]);
            }
    } else if (mode == AV1R_DC_PRED) {
        /* dcPredict (IntraPredict.cpp:485-508) */
        int avg, sum = 0;
        if (haveLeft && haveAbove) {
            for (int i = 0; i < hh; i++) sum += left[i];
            for (int j = 0; j < w; j++) sum += above[j];
            avg = (sum + ((w + hh) >> 1)) / (w + hh);
        } else if (haveLeft) {
            for (int i = 0; i < hh; i++) sum += left[i];
            avg = CLIP1((sum + (hh >> 1)) >> a->log2H);
        } else if (haveAbove) {
            for (int j = 0; j < w; j++) sum += above[j];
            avg = CLIP1((sum + (w >> 1)) >> a->log2W);
        } else {
            avg = 128;
        }
        for (int i = 0; i < hh; i++)
            for (int j = 0; j < w; j++)
                pred[i * 64 + j] = (uint8_t)avg;
    } else if (mode == AV1R_SMOOTH_PRED) {
        /* smoothPredict (IntraPredict.cpp:526-539) */
        const uint8_t* wx = sm_weights(a->log2W);
        const uint8_t* wy = sm_weights(a->log2H);
        for (int i = 0; i < hh; i++)
            for (int j = 0; j < w; j++) {
                int s = wy[i] * above[j] + (256 - wy[i]) * left[hh - 1] + wx[j] * left[i]
                    + (256 - wx[j]) * above[w - 1];
                pred[i * 64 + j] = (uint8_t)r2(s, 9);
            }
    } else if (mode == AV1R_SMOOTH_V_PRED) {
        const uint8_t* wy = sm_weights(a->log2H);
        for (int i = 0; i < hh; i++)
            for (int j = 0; j < w; j++)
                pred[i * 64 + j] = (uint8_t)r2(wy[i] * above[j] + (256 - wy[i]) * left[hh - 1], 8);
    } else if (mode == AV1R_SMOOTH_H_PRED) {
        const uint8_t* wx = sm_weights(a->log2W);
        for (int i = 0; i < hh; i++)
            for (int j = 0; j < w; j++)
                pred[i * 64 + j] = (uint8_t)r2(wx[j] * left[i] + (256 - wx[j]) * above[w - 1], 8);
    }
}

/* predict_chroma_from_luma (IntraPredict.cpp:632-667) */
static void predict_cfl(const oracle_ctx* c, const IntraArgs* a, uint8_t* pred)
{
    const OFrame* f = c->cur;
    int subX = c->h->subx, subY = c->h->suby;
    int w = 1 << a->log2W, hh = 1 << a->log2H;
    int alpha = a->plane == 1 ? a->blk->cfl_alpha_u : a->blk->cfl_alpha_v;
    int maxLW = a->blk->max_luma_w, maxLH = a->blk->max_luma_h;
    static _Thread_local int L[64 * 64];
    int avg = 0;
    for (int i = 0; i < hh; i++) {
        int ly = MIN((a->y + i) << subY, maxLH - (1 << subY));
        for (int j = 0; j < w; j++) {
            int lx = MIN((a->x + j) << subX, maxLW - (1 << subX));
            int t = 0;
            for (int dy = 0; dy <= subY; dy++)
                for (int dx = 0; dx <= subX; dx++)
                    t += PIX(f, 0, lx + dx, ly + dy);
            int v = t << (3 - subX - subY);
            L[i * 64 + j] = v;
            avg += v;
        }
    }
    avg = r2(avg, a->log2W + a->log2H);
    for (int i = 0; i < hh; i++)
        for (int j = 0; j < w; j++) {
            int dc = pred[i * 64 + j];
            int scaled = r2s(alpha * (L[i * 64 + j] - avg), 6);
            pred[i * 64 + j] = (uint8_t)CLIP1(dc + scaled);
        }
}

/* ======================================================================================
 * Inverse transforms (TransformBlock.cpp:1751-2253)
 * ==================================================================================== */
static int brev(int numBits, int x)
{
    int t = 0;
    for (int i = 0; i < numBits; i++)
        t |= ((x >> i) & 1) << (numBits - 1 - i);
    return t;
}
static int cos128(int angle)
{
    int a = angle & 255;
    if (a <= 64) return av1r_cos128[a];
    if (a <= 128) return -av1r_cos128[128 - a];
    if (a <= 192) return -av1r_cos128[a - 128];
    return av1r_cos128[256 - a];
}
static int sin128(int angle) { return cos128(angle - 64); }
/* butterfly B (TransformBlock.cpp:1799-1813) */
static void B(int* T, int a, int b, int angle, int flip)
{
    int x = T[a] * cos128(angle) - T[b] * sin128(angle);
    int y = T[a] * sin128(angle) + T[b] * cos128(angle);
    if (!flip) {
        T[a] = r2(x, 12);
        T[b] = r2(y, 12);
    } else {
        T[b] = r2(x, 12);
        T[a] = r2(y, 12);
    }
}
/* Hadamard H with clamp (TransformBlock.cpp:1815-1825) */
static void H(int* T, int a, int b, int flip, int r)
{
    if (flip) { int t = a; a = b; b = t; }
    int lo = -(1 << (r - 1)), hi = (1 << (r - 1)) - 1;
    int x = T[a], y = T[b];
    T[a] = CLIP3(lo, hi, x + y);
    T[b] = CLIP3(lo, hi, x - y);
}
/* iDct (TransformBlock.cpp:1827-1989) */
static void idct(int* T, int n, int r)
{
    int copy[64], cnt = 1 << n;
    memcpy(copy, T, sizeof(int) * cnt);
    for (int i = 0; i < cnt; i++) T[i] = copy[brev(n, i)];
    if (n == 6) for (int i = 0; i < 16; i++) B(T, 32 + i, 63 - i, 63 - 4 * brev(4, i), 0);
    if (n >= 5) for (int i = 0; i < 8; i++) B(T, 16 + i, 31 - i, 6 + (brev(3, 7 - i) << 3), 0);
    if (n == 6) for (int i = 0; i < 16; i++) H(T, 32 + i * 2, 33 + i * 2, i & 1, r);
    if (n >= 4) for (int i = 0; i < 4; i++) B(T, 8 + i, 15 - i, 12 + (brev(2, 3 - i) << 4), 0);
    if (n >= 5) for (int i = 0; i < 8; i++) H(T, 16 + 2 * i, 17 + 2 * i, i & 1, r);
    if (n == 6) for (int i = 0; i < 4; i++) for (int j = 0; j < 2; j++) B(T, 62 - i * 4 - j, 33 + i * 4 + j, 60 - 16 * brev(2, i) + 64 * j, 1);
    if (n >= 3) for (int i = 0; i < 2; i++) B(T, 4 + i, 7 - i, 56 - 32 * i, 0);
    if (n >= 4) for (int i = 0; i < 4; i++) H(T, 8 + 2 * i, 9 + 2 * i, i & 1, r);
    if (n >= 5) for (int i = 0; i < 2; i++) for (int j = 0; j < 2; j++) B(T, 30 - 4 * i - j, 17 + 4 * i + j, 24 + (j << 6) + ((1 - i) << 5), 1);
    if (n == 6) for (int i = 0; i < 8; i++) for (int j = 0; j < 2; j++) H(T, 32 + i * 4 + j, 35 + i * 4 - j, i & 1, r);
    for (int i = 0; i < 2; i++) B(T, 2 * i, 2 * i + 1, 32 + 16 * i, 1 - i);
    if (n >= 3) for (int i = 0; i < 2; i++) H(T, 4 + 2 * i, 5 + 2 * i, i, r);
    if (n >= 4) for (int i = 0; i < 2; i++) B(T, 14 - i, 9 + i, 48 + 64 * i, 1);
    if (n >= 5) for (int i = 0; i < 4; i++) for (int j = 0; j < 2; j++) H(T, 16 + 4 * i + j, 19 + 4 * i - j, i & 1, r);
    if (n == 6) for (int i = 0; i < 2; i++) for (int j = 0; j < 4; j++) B(T, 61 - i * 8 - j, 34 + i * 8 + j, 56 - i * 32 + (j >> 1) * 64, 1);
    for (int i = 0; i < 2; i++) H(T, i, 3 - i, 0, r);
    if (n >= 3) B(T, 6, 5, 32, 1);
    if (n >= 4) for (int i = 0; i < 2; i++) for (int j = 0; j < 2; j++) H(T, 8 + 4 * i + j, 11 + 4 * i - j, i, r);
    if (n >= 5) for (int i = 0; i < 4; i++) B(T, 29 - i, 18 + i, 48 + (i >> 1) * 64, 1);
    if (n == 6) for (int i = 0; i < 4; i++) for (int j = 0; j < 4; j++) H(T, 32 + 8 * i + j, 39 + 8 * i - j, i & 1, r);
    if (n >= 3) for (int i = 0; i < 4; i++) H(T, i, 7 - i, 0, r);
    if (n >= 4) for (int i = 0; i < 2; i++) B(T, 13 - i, 10 + i, 32, 1);
    if (n >= 5) for (int i = 0; i < 2; i++) for (int j = 0; j < 4; j++) H(T, 16 + i * 8 + j, 23 + i * 8 - j, i, r);
    if (n == 6) for (int i = 0; i < 8; i++) B(T, 59 - i, 36 + i, i < 4 ? 48 : 112, 1);
    if (n >= 4) for (int i = 0; i < 8; i++) H(T, i, 15 - i, 0, r);
    if (n >= 5) for (int i = 0; i < 4; i++) B(T, 27 - i, 20 + i, 32, 1);
    if (n == 6) for (int i = 0; i < 8; i++) { H(T, 32 + i, 47 - i, 0, r); H(T, 48 + i, 63 - i, 1, r); }
    if (n >= 5) for (int i = 0; i < 16; i++) H(T, i, 31 - i, 0, r);
    if (n == 6) {
        for (int i = 0; i < 8; i++) B(T, 55 - i, 40 + i, 32, 1);
        for (int i = 0; i < 32; i++) H(T, i, 63 - i, 0, r);
    }
}
/* iAdst4 (TransformBlock.cpp:1991-2027) */
static void iadst4(int* T)
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
    int x0 = s0 + s3, x1 = s1 + s3, x2 = s2, x3 = s0 + s1;
    x3 = x3 - s3;
    T[0] = r2(x0, 12);
    T[1] = r2(x1, 12);
    T[2] = r2(x2, 12);
    T[3] = r2(x3, 12);
}
static void adst_in_perm(int* T, int n)
{
    int n0 = 1 << n, copy[16];
    memcpy(copy, T, sizeof(int) * n0);
    for (int i = 0; i < n0; i++)
        T[i] = copy[(i & 1) ? (i - 1) : (n0 - i - 1)];
}
static void adst_out_perm(int* T, int n)
{
    int n0 = 1 << n, copy[16];
    memcpy(copy, T, sizeof(int) * n0);
    for (int i = 0; i < n0; i++) {
        int a = (i >> 3) & 1;
        int b = ((i >> 2) & 1) ^ ((i >> 3) & 1);
        int c = ((i >> 1) & 1) ^ ((i >> 2) & 1);
        int d = (i & 1) ^ ((i >> 1) & 1);
        int idx = ((d << 3) | (c << 2) | (b << 1) | a) >> (4 - n);
        T[i] = (i & 1) ? -copy[idx] : copy[idx];
    }
}
/* iAdst8 / iAdst16 (TransformBlock.cpp:2056-2112) */
static void iadst8(int* T, int r)
{
    adst_in_perm(T, 3);
    for (int i = 0; i < 4; i++) B(T, 2 * i, 2 * i + 1, 60 - 16 * i, 1);
    for (int i = 0; i < 4; i++) H(T, i, 4 + i, 0, r);
    for (int i = 0; i < 2; i++) B(T, 4 + 3 * i, 5 + i, 48 - 32 * i, 1);
    for (int i = 0; i < 2; i++) for (int j = 0; j < 2; j++) H(T, 4 * j + i, 2 + 4 * j + i, 0, r);
    for (int i = 0; i < 2; i++) B(T, 2 + 4 * i, 3 + 4 * i, 32, 1);
    adst_out_perm(T, 3);
}
static void iadst16(int* T, int r)
{
    adst_in_perm(T, 4);
    for (int i = 0; i < 8; i++) B(T, 2 * i, 2 * i + 1, 62 - 8 * i, 1);
    for (int i = 0; i < 8; i++) H(T, i, 8 + i, 0, r);
    for (int i = 0; i < 2; i++) { B(T, 8 + 2 * i, 9 + 2 * i, 56 - 32 * i, 1); B(T, 13 + 2 * i, 12 + 2 * i, 8 + 32 * i, 1); }
    for (int i = 0; i < 4; i++) for (int j = 0; j < 2; j++) H(T, 8 * j + i, 4 + 8 * j + i, 0, r);
    for (int i = 0; i < 2; i++) for (int j = 0; j < 2; j++) B(T, 4 + 8 * j + 3 * i, 5 + 8 * j + i, 48 - 32 * i, 1);
    for (int i = 0; i < 2; i++) for (int j = 0; j < 4; j++) H(T, 4 * j + i, 2 + 4 * j + i, 0, r);
    for (int i = 0; i < 4; i++) B(T, 2 + 4 * i, 3 + 4 * i, 32, 1);
    adst_out_perm(T, 4);
}
static void iadst(int* T, int n, int r)
{
    if (n == 2) iadst4(T);
    else if (n == 3) iadst8(T, r);
    else if (n == 4) iadst16(T, r);
}
/* iIdentity (TransformBlock.cpp:2127-2147) */
static void iidentity(int* T, int n)
{
    int size = 1 << n;
    for (int i = 0; i < size; i++) {
        if (n == 2) T[i] = r2(T[i] * 5793, 12);
        else if (n == 3) T[i] = T[i] * 2;
        else if (n == 4) T[i] = r2(T[i] * 11586, 12);
        else if (n == 5) T[i] = T[i] * 4;
    }
}
/* inverseWalshHadamardTransform (TransformBlock.cpp:2149-2166) */
static void iwht(int* T, int shift)
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
static int row_is_dct(int t) { return t == AV1R_DCT_DCT || t == AV1R_ADST_DCT || t == AV1R_FLIPADST_DCT || t == AV1R_H_DCT; }
static int row_is_adst(int t)
{
    return t == AV1R_DCT_ADST || t == AV1R_ADST_ADST || t == AV1R_DCT_FLIPADST || t == AV1R_FLIPADST_FLIPADST
        || t == AV1R_ADST_FLIPADST || t == AV1R_FLIPADST_ADST || t == AV1R_H_ADST || t == AV1R_H_FLIPADST;
}
static int col_is_dct(int t) { return t == AV1R_DCT_DCT || t == AV1R_DCT_ADST || t == AV1R_DCT_FLIPADST || t == AV1R_V_DCT; }
static int col_is_adst(int t)
{
    return t == AV1R_ADST_DCT || t == AV1R_ADST_ADST || t == AV1R_FLIPADST_DCT || t == AV1R_FLIPADST_FLIPADST
        || t == AV1R_ADST_FLIPADST || t == AV1R_FLIPADST_ADST || t == AV1R_V_ADST || t == AV1R_V_FLIPADST;
}

/* reconstruct (TransformBlock.cpp:2255-2276) + inverseTransform (:2173-2253).
 * Writes Residual[h][w] (row stride 64). */
static void reconstruct(const oracle_ctx* c, const av1r_tb* tb, const av1r_block* blk, int* res)
{
    int txSz = tb->tx_size;
    int w = av1r_tx_w[txSz], hh = av1r_tx_h[txSz];
    int log2W = av1r_tx_w_log2[txSz], log2H = av1r_tx_h_log2[txSz];
    if (!tb->coef_cnt) {
        for (int i = 0; i < hh; i++) memset(res + i * 64, 0, w * sizeof(int));
        return;
    }
    const av1r_frame_hdr* h = c->h;
    int tw = MIN(w, 32), th = MIN(hh, 32);
    int dqDenom = 1;
    if (txSz == AV1R_TX_32X32 || txSz == AV1R_TX_16X32 || txSz == AV1R_TX_32X16 || txSz == AV1R_TX_16X64 || txSz == AV1R_TX_64X16)
        dqDenom = 2;
    else if (txSz == AV1R_TX_64X64 || txSz == AV1R_TX_32X64 || txSz == AV1R_TX_64X32)
        dqDenom = 4;
    /* get_dc_quant / get_ac_quant (TransformBlock.cpp:1706-1728): segmentation is not
     * supported (README), so qindex is the block's get_qindex() value. */
    int dcDelta = tb->plane == 0 ? h->delta_q_y_dc : tb->plane == 1 ? h->delta_q_u_dc : h->delta_q_v_dc;
    int acDelta = tb->plane == 0 ? 0 : tb->plane == 1 ? h->delta_q_u_ac : h->delta_q_v_ac;
    int dcQ = av1r_dc_qlookup[CLIP3(0, 255, blk->qindex + dcDelta)];
    int acQ = av1r_ac_qlookup[CLIP3(0, 255, blk->qindex + acDelta)];
    static _Thread_local int dq[32 * 32];
    memset(dq, 0, sizeof(dq));
    const uint32_t* cf = c->b->coefs + tb->coef_off;
    for (int k = 0; k < tb->coef_cnt; k++) {
        int pos = AV1R_COEF_POS(cf[k]);
        int level = AV1R_COEF_LEVEL(cf[k]);
        int q = pos == 0 ? dcQ : acQ;
        int d = (int)((uint32_t)level * (uint32_t)q); /* int multiply as the reference (wraps) */
        int sign = d < 0 ? -1 : 1;
        int d2 = sign * (iabs(d) & 0xffffff) / dqDenom;
        dq[(pos / tw) * 32 + (pos % tw)] = CLIP3(-(1 << 15), (1 << 15) - 1, d2);
    }
    (void)th;
    int lossless = (blk->flags & AV1R_BLK_LOSSLESS) != 0;
    int type = tb->tx_type;
    int rowShift = lossless ? 0 : av1r_tx_row_shift[txSz];
    int colShift = lossless ? 0 : 4;
    int rowClamp = 16; /* BitDepth + 8 */
    int colClamp = 16; /* max(BitDepth + 6, 16) */
    int lo = -(1 << (colClamp - 1)), hi = (1 << (colClamp - 1)) - 1;
    int T[64];
    for (int i = 0; i < hh; i++) {
        for (int j = 0; j < w; j++)
            T[j] = (i < 32 && j < 32) ? dq[i * 32 + j] : 0;
        if (iabs(log2W - log2H) == 1)
            for (int j = 0; j < w; j++) T[j] = r2(T[j] * 2896, 12);
        if (lossless) iwht(T, 2);
        else if (row_is_dct(type)) idct(T, log2W, rowClamp);
        else if (row_is_adst(type)) iadst(T, log2W, rowClamp);
        else iidentity(T, log2W);
        for (int j = 0; j < w; j++)
            res[i * 64 + j] = CLIP3(lo, hi, r2(T[j], rowShift));
    }
    for (int j = 0; j < w; j++) {
        for (int i = 0; i < hh; i++) T[i] = res[i * 64 + j];
        if (lossless) iwht(T, 0);
        else if (col_is_dct(type)) idct(T, log2H, colClamp);
        else if (col_is_adst(type)) iadst(T, log2H, colClamp);
        else iidentity(T, log2H);
        for (int i = 0; i < hh; i++) res[i * 64 + j] = r2(T[i], colShift);
    }
}

/* TransformBlock::decode (TransformBlock.cpp:2376-2456) */
static void decode_tb(oracle_ctx* c, const av1r_tb* tb)
{
    const av1r_block* blk = &c->b->blocks[tb->block];
    OFrame* f = c->cur;
    int plane = tb->plane, x = tb->x, y = tb->y, txSz = tb->tx_size;
    int w = av1r_tx_w[txSz], hh = av1r_tx_h[txSz];
    int isInter = (blk->flags & AV1R_BLK_INTER) != 0;
    int palSize = plane ? blk->palette_size_uv : blk->palette_size_y;
    static _Thread_local uint8_t pred[64 * 64];
    static _Thread_local int res[64 * 64];
    if (!isInter) {
        if (palSize) {
            /* Block::Palette::predict_palette (Block.cpp:2279-2298) */
            const uint8_t* ph = c->b->palette + blk->palette_off;
            int subX = plane ? c->h->subx : 0, subY = plane ? c->h->suby : 0;
            int bx = x - (blk->mi_col >> subX) * 4, by = y - (blk->mi_row >> subY) * 4;
            int mw = plane ? ph[2] : ph[0];
            const uint8_t* map = ph + AV1R_PALETTE_HDR + (plane ? ph[0] * ph[1] : 0);
            const uint8_t* colors = ph + 4 + 8 * plane;
            for (int i = 0; i < hh; i++)
                for (int j = 0; j < w; j++)
                    PIX(f, plane, x + j, y + i) = colors[map[(by + i) * mw + bx + j]];
        } else {
            IntraArgs a = {plane, x, y, av1r_tx_w_log2[txSz], av1r_tx_h_log2[txSz], blk};
            int isCfl = plane > 0 && blk->uv_mode == AV1R_UV_CFL_PRED;
            int mode = plane == 0 ? blk->y_mode : (isCfl ? AV1R_DC_PRED : blk->uv_mode);
            predict_intra(c, &a, tb->flags & AV1R_TB_HAVE_LEFT ? 1 : 0, tb->flags & AV1R_TB_HAVE_ABOVE ? 1 : 0,
                tb->flags & AV1R_TB_HAVE_AR ? 1 : 0, tb->flags & AV1R_TB_HAVE_BL ? 1 : 0, mode, pred);
            if (isCfl)
                predict_cfl(c, &a, pred);
        }
    }
    reconstruct(c, tb, blk, res);
    int t = tb->tx_type;
    int flipUD = t == AV1R_FLIPADST_DCT || t == AV1R_FLIPADST_ADST || t == AV1R_V_FLIPADST || t == AV1R_FLIPADST_FLIPADST;
    int flipLR = t == AV1R_DCT_FLIPADST || t == AV1R_ADST_FLIPADST || t == AV1R_H_FLIPADST || t == AV1R_FLIPADST_FLIPADST;
    if (!tb->coef_cnt)
        flipUD = flipLR = 0;
    for (int i = 0; i < hh; i++)
        for (int j = 0; j < w; j++) {
            int xx = flipLR ? (w - j - 1) : j;
            int yy = flipUD ? (hh - i - 1) : i;
            int p = (!isInter && !palSize) ? pred[i * 64 + j] : PIX(f, plane, x + j, y + i);
            PIX(f, plane, x + j, y + i) = (uint8_t)CLIP1(res[yy * 64 + xx] + p);
        }
}

/* ======================================================================================
 * Inter prediction (InterPredict.cpp:34-1049)
 * ==================================================================================== */
typedef struct Inter {
    oracle_ctx* c;
    const av1r_block* blk;
    int plane, subX, subY;
    int isCompound, R0, R1, PostRound;
    int startX, startY, xStep, yStep;
} Inter;

/* Block::LocalWarp::resolveDivisor (Block.cpp:1087-1095) */
static void resolve_divisor(int64_t d, int* divShift, int* divFactor)
{
    int64_t ad = d < 0 ? -d : d;
    int n = floor_log2(ad);
    int64_t e = ad - ((int64_t)1 << n);
    int64_t f = n > 8 ? r2_64(e, n - 8) : (e << (8 - n));
    *divShift = n + 14;
    *divFactor = d < 0 ? -(int)av1r_div_lut[f] : (int)av1r_div_lut[f];
}
/* Block::LocalWarp::setupShear (Block.cpp:1179-1200) */
static int setup_shear(const int32_t* wp, int* alpha, int* beta, int* gamma, int* delta)
{
    int alpha0 = CLIP3(-32768, 32767, wp[2] - (1 << 16));
    int beta0 = CLIP3(-32768, 32767, wp[3]);
    int divShift, divFactor;
    resolve_divisor(wp[2], &divShift, &divFactor);
    int64_t v = (int64_t)(wp[4] << 16);
    int gamma0 = CLIP3(-32768, 32767, (int)r2s_64(v * divFactor, divShift));
    int64_t w = (int64_t)(wp[3] * wp[4]);
    int delta0 = CLIP3(-32768, 32767, wp[5] - (int)r2s_64(w * divFactor, divShift) - (1 << 16));
    *alpha = r2s(alpha0, 6) << 6;
    *beta = r2s(beta0, 6) << 6;
    *gamma = r2s(gamma0, 6) << 6;
    *delta = r2s(delta0, 6) << 6;
    if ((4 * iabs(*alpha) + 7 * iabs(*beta)) >= (1 << 16)) return 0;
    if ((4 * iabs(*gamma) + 4 * iabs(*delta)) >= (1 << 16)) return 0;
    return 1;
}

static const OFrame* ref_frame(const Inter* I, int refIdx)
{
    return refIdx < 0 ? I->c->cur : I->c->store[refIdx];
}
/* getScale (Parser.cpp:788-793) */
static void get_scale(const Inter* I, int refIdx, int* xs, int* ys)
{
    const av1r_frame_hdr* h = I->c->h;
    int rw = refIdx < 0 ? h->frame_width : I->c->store[refIdx]->width;
    int rh = refIdx < 0 ? h->frame_height : I->c->store[refIdx]->height;
    *xs = ((rw << 14) + (h->frame_width / 2)) / h->frame_width;
    *ys = ((rh << 14) + (h->frame_height / 2)) / h->frame_height;
}
/* motionVectorScaling (InterPredict.cpp:66-83) */
static void mv_scaling(Inter* I, int refIdx, int x, int y, const int16_t* mv)
{
    int xs, ys;
    get_scale(I, refIdx, &xs, &ys);
    int origX = ((x << 4) + ((2 * mv[1]) >> I->subX) + 8);
    int origY = ((y << 4) + ((2 * mv[0]) >> I->subY) + 8);
    int baseX = (origX * xs - (8 << 14));
    int baseY = (origY * ys - (8 << 14));
    I->startX = r2s(baseX, 14 + 4 - 10) + 32;
    I->startY = r2s(baseY, 14 + 4 - 10) + 32;
    I->xStep = r2s(xs, 14 - 10);
    I->yStep = r2s(ys, 14 - 10);
}
/* getFilterIdx (InterPredict.cpp:85-97) */
static int filter_idx(const av1r_mi* info, int size, int dir)
{
    int f = dir ? (info->filt >> 4) : (info->filt & 15);
    if (size <= 4) {
        if (f == AV1R_EIGHTTAP || f == AV1R_EIGHTTAP_SHARP) return 4;
        if (f == AV1R_EIGHTTAP_SMOOTH) return 5;
    }
    return f;
}
/* blockInterPrediction (InterPredict.cpp:385-402) with blockPixelPredict (:319-331) and
 * blockSubPixelPredict (:333-383) */
static void block_inter_pred(Inter* I, int refIdx, int refList, int w, int h, int candRow, int candCol)
{
    oracle_ctx* c = I->c;
    int16_t (*pred)[128] = c->preds[refList];
    const OFrame* ref = ref_frame(I, refIdx);
    int plane = I->plane;
    int lastX, lastY;
    if (refIdx < 0) {
        lastX = ((c->h->mi_cols * 4 + I->subX) >> I->subX) - 1;
        lastY = ((c->h->mi_rows * 4 + I->subY) >> I->subY) - 1;
    } else {
        lastX = ((ref->width + I->subX) >> I->subX) - 1;
        lastY = ((ref->height + I->subY) >> I->subY) - 1;
    }
    if (!((I->startX >> 6) & 15) && !((I->startY >> 6) & 15)) {
        int x = I->startX >> 10, y = I->startY >> 10;
        for (int r = 0; r < h; r++)
            for (int cc = 0; cc < w; cc++)
                pred[r][cc] = (int16_t)(PIX(ref, plane, CLIP3(0, lastX, x + cc), CLIP3(0, lastY, y + r))
                    << (14 - I->R0 - I->R1));
        return;
    }
    const av1r_mi* info = mi_at(c, candRow, candCol);
    int ih = (((h - 1) * I->yStep + (1 << 10) - 1) >> 10) + 8;
    static _Thread_local int inter[136][128];
    int fidx = filter_idx(info, w, 1);
    for (int r = 0; r < ih; r++) {
        int y = CLIP3(0, lastY, (I->startY >> 10) + r - 3);
        for (int cc = 0; cc < w; cc++) {
            int p = I->startX + I->xStep * cc;
            const int16_t* flt = av1r_subpel_filters + (fidx * 16 + ((p >> 6) & 15)) * 8;
            int x = (p >> 10) - 3;
            int s = 0;
            for (int t = 0; t < 8; t++)
                s += flt[t] * PIX(ref, plane, CLIP3(0, lastX, x + t), y);
            inter[r][cc] = r2(s, I->R0);
        }
    }
    fidx = filter_idx(info, h, 0);
    for (int r = 0; r < h; r++)
        for (int cc = 0; cc < w; cc++) {
            int p = (I->startY & 1023) + I->yStep * r;
            const int16_t* flt = av1r_subpel_filters + (fidx * 16 + ((p >> 6) & 15)) * 8;
            int y = p >> 10;
            int s = 0;
            for (int t = 0; t < 8; t++)
                s += flt[t] * inter[y + t][cc];
            pred[r][cc] = (int16_t)r2(s, I->R1);
        }
}
/* blockWarp (InterPredict.cpp:507-553) */
static void block_warp(Inter* I, const int32_t* wp, int refIdx, int refList, int x, int y, int i8, int j8, int w, int h)
{
    oracle_ctx* c = I->c;
    const OFrame* ref = c->store[refIdx];
    int16_t (*pred)[128] = c->preds[refList];
    int plane = I->plane;
    int lastX = ((ref->width + I->subX) >> I->subX) - 1;
    int lastY = ((ref->height + I->subY) >> I->subY) - 1;
    int srcX = (x + j8 * 8 + 4) << I->subX;
    int srcY = (y + i8 * 8 + 4) << I->subY;
    int dstX = wp[2] * srcX + wp[3] * srcY + wp[0];
    int dstY = wp[4] * srcX + wp[5] * srcY + wp[1];
    int alpha, beta, gamma, delta;
    setup_shear(wp, &alpha, &beta, &gamma, &delta);
    int inter[16][8];
    int x4 = dstX >> I->subX, y4 = dstY >> I->subY;
    int ix4 = x4 >> 16, sx4 = x4 & 0xffff, iy4 = y4 >> 16, sy4 = y4 & 0xffff;
    for (int i1 = -7; i1 < 8; i1++)
        for (int i2 = -4; i2 < 4; i2++) {
            int sx = sx4 + alpha * i2 + beta * i1;
            int offs = r2(sx, 10) + 64;
            int s = 0;
            for (int i3 = 0; i3 < 8; i3++)
                s += av1r_warped_filters[offs * 8 + i3]
                    * PIX(ref, plane, CLIP3(0, lastX, ix4 + i2 - 3 + i3), CLIP3(0, lastY, iy4 + i1));
            inter[i1 + 7][i2 + 4] = r2(s, I->R0);
        }
    for (int i1 = -4; i1 < MIN(4, h - i8 * 8 - 4); i1++)
        for (int i2 = -4; i2 < MIN(4, w - j8 * 8 - 4); i2++) {
            int sy = sy4 + gamma * i2 + delta * i1;
            int offs = r2(sy, 10) + 64;
            int s = 0;
            for (int i3 = 0; i3 < 8; i3++)
                s += av1r_warped_filters[offs * 8 + i3] * inter[i1 + i3 + 4][i2 + 4];
            pred[i8 * 8 + i1 + 4][j8 * 8 + i2 + 4] = (int16_t)r2(s, I->R1);
        }
}

/* initialise_wedge_mask_table (InterPredict.cpp:835-886): built once. */
/* per thread: oracle instances may run concurrently (tests drive one per stream) */
static _Thread_local uint8_t g_master[6][64][64];
static _Thread_local uint8_t g_wedge_flip[AV1R_BLOCK_SIZES][16];
static _Thread_local int g_wedge_init;
static void wedge_init(void)
{
    if (g_wedge_init) return;
    for (int j = 0; j < 64; j++) {
        int shift = 16;
        for (int i = 0; i < 64; i += 2) {
            g_master[AV1R_WEDGE_OBLIQUE63][i][j] = av1r_wedge_master_oblique_even[CLIP3(0, 63, j - shift)];
            shift -= 1;
            g_master[AV1R_WEDGE_OBLIQUE63][i + 1][j] = av1r_wedge_master_oblique_odd[CLIP3(0, 63, j - shift)];
            g_master[AV1R_WEDGE_VERTICAL][i][j] = av1r_wedge_master_vertical[j];
            g_master[AV1R_WEDGE_VERTICAL][i + 1][j] = av1r_wedge_master_vertical[j];
        }
    }
    for (int i = 0; i < 64; i++)
        for (int j = 0; j < 64; j++) {
            int msk = g_master[AV1R_WEDGE_OBLIQUE63][i][j];
            g_master[AV1R_WEDGE_OBLIQUE27][j][i] = (uint8_t)msk;
            g_master[AV1R_WEDGE_OBLIQUE117][i][63 - j] = (uint8_t)(64 - msk);
            g_master[AV1R_WEDGE_OBLIQUE153][63 - j][i] = (uint8_t)(64 - msk);
            g_master[AV1R_WEDGE_HORIZONTAL][j][i] = g_master[AV1R_WEDGE_VERTICAL][i][j];
        }
    for (int bs = AV1R_BLOCK_8X8; bs < AV1R_BLOCK_SIZES; bs++) {
        if (!av1r_wedge_bits[bs]) continue;
        int w = av1r_num4x4w[bs] * 4, h = av1r_num4x4h[bs] * 4;
        int shape = h > w ? 0 : (h < w ? 1 : 2);
        for (int wedge = 0; wedge < 16; wedge++) {
            const uint8_t* cb = av1r_wedge_codebook[shape][wedge];
            int xoff = 32 - ((cb[1] * w) >> 3), yoff = 32 - ((cb[2] * h) >> 3);
            int sum = 0;
            for (int i = 0; i < w; i++) sum += g_master[cb[0]][yoff][xoff + i];
            for (int i = 1; i < h; i++) sum += g_master[cb[0]][yoff + i][xoff];
            int avg = (sum + (w + h - 1) / 2) / (w + h - 1);
            g_wedge_flip[bs][wedge] = avg < 32;
        }
    }
    g_wedge_init = 1;
}
/* WedgeMasks[bsize][sign][wedge][i][j] */
static int wedge_mask_at(int bs, int sign, int wedge, int i, int j)
{
    int w = av1r_num4x4w[bs] * 4, h = av1r_num4x4h[bs] * 4;
    int shape = h > w ? 0 : (h < w ? 1 : 2);
    const uint8_t* cb = av1r_wedge_codebook[shape][wedge];
    int xoff = 32 - ((cb[1] * w) >> 3), yoff = 32 - ((cb[2] * h) >> 3);
    int m = g_master[cb[0]][yoff + i][xoff + j];
    return sign == g_wedge_flip[bs][wedge] ? m : 64 - m;
}

/* getDistanceWeights (InterPredict.cpp:917-960) */
static void distance_weights(const Inter* I, int candRow, int candCol, int* fwd, int* bck)
{
    const av1r_mi* info = mi_at(I->c, candRow, candCol);
    int dist[2];
    for (int l = 0; l < 2; l++) {
        int ref = info->ref_frame[l];
        dist[l] = I->c->h->ref_dist[ref & 7];
    }
    int d0 = dist[1], d1 = dist[0];
    int order = d0 <= d1;
    if (d0 == 0 || d1 == 0) {
        *fwd = av1r_quant_dist_lookup[3][order];
        *bck = av1r_quant_dist_lookup[3][1 - order];
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
    *fwd = av1r_quant_dist_lookup[i][order];
    *bck = av1r_quant_dist_lookup[i][1 - order];
}

/* predict_overlap (InterPredict.cpp:611-628) */
static void predict_overlap(Inter* I, int pass, int candRow, int candCol, int x4, int y4, int predW, int predH, const uint8_t* mask)
{
    oracle_ctx* c = I->c;
    const av1r_mi* info = mi_at(c, candRow, candCol);
    int refIdx = c->h->ref_frame_idx[info->ref_frame[0] - 1];
    int predX = (x4 * 4) >> I->subX, predY = (y4 * 4) >> I->subY;
    mv_scaling(I, refIdx, predX, predY, info->mv[0]);
    block_inter_pred(I, refIdx, 0, predW, predH, candRow, candCol);
    OFrame* f = c->cur;
    for (int i = 0; i < predH; i++)
        for (int j = 0; j < predW; j++) {
            int m = pass ? mask[j] : mask[i];
            int px = PIX(f, I->plane, predX + j, predY + i);
            PIX(f, I->plane, predX + j, predY + i) = (uint8_t)CLIP1(r2(m * px + (64 - m) * CLIP1(c->preds[0][i][j]), 6));
        }
}
static const uint8_t* obmc_mask(int len)
{
    return av1r_obmc_mask + (len == 2 ? 0 : len == 4 ? 2 : len == 8 ? 6 : len == 16 ? 14 : 30);
}
/* overlappedMotionCompensation (InterPredict.cpp:658-709) */
static void obmc(Inter* I, int w, int h)
{
    oracle_ctx* c = I->c;
    const av1r_block* blk = I->blk;
    int bs = blk->mi_size;
    if (blk->flags & AV1R_BLK_AVAIL_U) {
        if (plane_size(bs, I->plane) >= AV1R_BLOCK_8X8) {
            int w4 = av1r_num4x4w[bs], x4 = blk->mi_col, y4 = blk->mi_row;
            int nCount = 0, nLimit = MIN(4, av1r_miw_log2[bs]);
            while (nCount < nLimit && x4 < MIN(c->h->mi_cols, blk->mi_col + w4)) {
                int candRow = blk->mi_row - 1, candCol = x4 | 1;
                const av1r_mi* info = mi_at(c, candRow, candCol);
                int step4 = CLIP3(2, 16, av1r_num4x4w[info->mi_size]);
                if (info->ref_frame[0] > AV1R_INTRA_FRAME) {
                    nCount++;
                    int predW = MIN(w, (step4 * 4) >> I->subX);
                    int predH = MIN(h >> 1, 32 >> I->subY);
                    predict_overlap(I, 0, candRow, candCol, x4, y4, predW, predH, obmc_mask(predH));
                }
                x4 += step4;
            }
        }
    }
    if (blk->flags & AV1R_BLK_AVAIL_L) {
        int h4 = av1r_num4x4h[bs], x4 = blk->mi_col, y4 = blk->mi_row;
        int nCount = 0, nLimit = MIN(4, av1r_mih_log2[bs]);
        while (nCount < nLimit && y4 < MIN(c->h->mi_rows, blk->mi_row + h4)) {
            int candCol = blk->mi_col - 1, candRow = y4 | 1;
            const av1r_mi* info = mi_at(c, candRow, candCol);
            int step4 = CLIP3(2, 16, av1r_num4x4h[info->mi_size]);
            if (info->ref_frame[0] > AV1R_INTRA_FRAME) {
                nCount++;
                int predW = MIN(w >> 1, 32 >> I->subX);
                int predH = MIN(h, (step4 * 4) >> I->subY);
                predict_overlap(I, 1, candRow, candCol, x4, y4, predW, predH, obmc_mask(predW));
            }
            y4 += step4;
        }
    }
}

/* predict_inter (InterPredict.cpp:962-1049) */
static void predict_inter(oracle_ctx* c, const av1r_block* blk, int plane, int x, int y, int w, int h, int candRow, int candCol)
{
    const av1r_frame_hdr* hd = c->h;
    Inter I;
    memset(&I, 0, sizeof(I));
    I.c = c;
    I.blk = blk;
    I.plane = plane;
    I.subX = plane ? hd->subx : 0;
    I.subY = plane ? hd->suby : 0;
    const av1r_mi* info = mi_at(c, candRow, candCol);
    I.isCompound = info->ref_frame[1] > AV1R_INTRA_FRAME;
    I.R0 = 3;
    I.R1 = I.isCompound ? 7 : 11;
    I.PostRound = 14 - (I.R0 + I.R1);
    int globalValid = 0;
    int isIntrabc = (blk->flags & AV1R_BLK_INTRABC) != 0;
    for (int refList = 0; refList < 1 + I.isCompound; refList++) {
        int refFrame = info->ref_frame[refList];
        int isGlobalMode = blk->y_mode == AV1R_GLOBALMV || blk->y_mode == AV1R_GLOBAL_GLOBALMV;
        if (isGlobalMode && hd->gm_type[refFrame & 7] > AV1R_GM_TRANSLATION) {
            int al, be, ga, de;
            globalValid = setup_shear(hd->gm_params[refFrame & 7], &al, &be, &ga, &de);
        }
        int refIdx = isIntrabc ? -1 : hd->ref_frame_idx[refFrame - 1];
        /* getUseWarp (InterPredict.cpp:50-64) */
        int useWarp = 0;
        if (!(w < 8 || h < 8) && !hd->force_integer_mv) {
            if (blk->motion_mode == AV1R_LOCALWARP && (blk->flags & AV1R_BLK_LOCAL_VALID)) {
                useWarp = 1;
            } else if (isGlobalMode && hd->gm_type[refFrame & 7] > AV1R_GM_TRANSLATION && globalValid) {
                int xs, ys;
                get_scale(&I, refIdx, &xs, &ys);
                if (xs == (1 << 14) && ys == (1 << 14))
                    useWarp = 2;
            }
        }
        mv_scaling(&I, refIdx, x, y, info->mv[refList]);
        if (useWarp) {
            const int32_t* wp = useWarp == 1 ? blk->local_warp : hd->gm_params[refFrame & 7];
            for (int i8 = 0; i8 <= ((h - 1) >> 3); i8++)
                for (int j8 = 0; j8 <= ((w - 1) >> 3); j8++)
                    block_warp(&I, wp, refIdx, refList, x, y, i8, j8, w, h);
        } else {
            block_inter_pred(&I, refIdx, refList, w, h, candRow, candCol);
        }
    }
    int ct = blk->compound_type;
    int isII = (blk->flags & AV1R_BLK_INTER) && mi_at(c, blk->mi_row, blk->mi_col)->ref_frame[1] == AV1R_INTRA_FRAME;
    if (ct == AV1R_COMPOUND_WEDGE) {
        /* wedgeMask (InterPredict.cpp:888-899) */
        wedge_init();
        int mw = w << I.subX, mh = h << I.subY;
        for (int i = 0; i < mh; i++)
            for (int j = 0; j < mw; j++)
                c->mask[i][j] = (uint8_t)wedge_mask_at(blk->mi_size, blk->wedge_sign, blk->wedge_index, i, j);
    } else if (ct == AV1R_COMPOUND_INTRA) {
        /* intraModeVariantMask (InterPredict.cpp:555-582) */
        int sizeScale = 128 / MAX(h, w);
        for (int i = 0; i < h; i++)
            for (int j = 0; j < w; j++) {
                int m = 32;
                if (blk->interintra_mode == AV1R_II_V_PRED) m = av1r_ii_weights_1d[i * sizeScale];
                else if (blk->interintra_mode == AV1R_II_H_PRED) m = av1r_ii_weights_1d[j * sizeScale];
                else if (blk->interintra_mode == AV1R_II_SMOOTH_PRED) m = av1r_ii_weights_1d[MIN(i, j) * sizeScale];
                c->mask[i][j] = (uint8_t)m;
            }
    } else if (ct == AV1R_COMPOUND_DIFFWTD && plane == 0) {
        /* differenceWeightMask (InterPredict.cpp:901-915) */
        for (int i = 0; i < h; i++)
            for (int j = 0; j < w; j++) {
                int16_t diff = (int16_t)iabs(c->preds[0][i][j] - c->preds[1][i][j]);
                diff = (int16_t)r2(diff, I.PostRound);
                int m = CLIP3(0, 64, 38 + diff / 16);
                c->mask[i][j] = (uint8_t)(blk->mask_type ? 64 - m : m);
            }
    }
    OFrame* f = c->cur;
    if (!I.isCompound && !isII) {
        for (int i = 0; i < h; i++)
            for (int j = 0; j < w; j++)
                PIX(f, plane, x + j, y + i) = (uint8_t)CLIP1(c->preds[0][i][j]);
    } else if (ct == AV1R_COMPOUND_AVERAGE) {
        for (int i = 0; i < h; i++)
            for (int j = 0; j < w; j++)
                PIX(f, plane, x + j, y + i) = (uint8_t)CLIP1(r2(c->preds[0][i][j] + c->preds[1][i][j], 1 + I.PostRound));
    } else if (ct == AV1R_COMPOUND_DISTANCE) {
        int fwd, bck;
        distance_weights(&I, candRow, candCol, &fwd, &bck);
        for (int i = 0; i < h; i++)
            for (int j = 0; j < w; j++)
                PIX(f, plane, x + j, y + i) = (uint8_t)CLIP1(r2(fwd * c->preds[0][i][j] + bck * c->preds[1][i][j], 4 + I.PostRound));
    } else {
        /* maskBlend (InterPredict.cpp:584-609) */
        int ii = (blk->flags & AV1R_BLK_INTERINTRA) != 0;
        int wii = (blk->flags & AV1R_BLK_WEDGE_II) != 0;
        for (int yy = 0; yy < h; yy++)
            for (int xx = 0; xx < w; xx++) {
                int m;
                if ((!I.subX && !I.subY) || (ii && !wii)) m = c->mask[yy][xx];
                else if (I.subX && !I.subY) m = r2(c->mask[yy][2 * xx] + c->mask[yy][2 * xx + 1], 1);
                else if (!I.subX && I.subY) m = r2(c->mask[2 * yy][xx] + c->mask[2 * yy + 1][xx], 1);
                else m = r2(c->mask[2 * yy][2 * xx] + c->mask[2 * yy][2 * xx + 1] + c->mask[2 * yy + 1][2 * xx] + c->mask[2 * yy + 1][2 * xx + 1], 2);
                if (ii) {
                    int p0 = CLIP1(r2(c->preds[0][yy][xx], I.PostRound));
                    int p1 = PIX(f, plane, x + xx, y + yy);
                    PIX(f, plane, x + xx, y + yy) = (uint8_t)CLIP1(r2(m * p1 + (64 - m) * p0, 6));
                } else {
                    PIX(f, plane, x + xx, y + yy) = (uint8_t)CLIP1(r2(m * c->preds[0][yy][xx] + (64 - m) * c->preds[1][yy][xx], 6 + I.PostRound));
                }
            }
    }
    if (blk->motion_mode == AV1R_OBMC_CAUSAL)
        obmc(&I, w, h);
}

/* Block::compute_prediction (Block.cpp:100-174) */
static void compute_prediction(oracle_ctx* c, const av1r_block* blk)
{
    const av1r_frame_hdr* hd = c->h;
    int isInter = (blk->flags & AV1R_BLK_INTER) != 0;
    int hasChroma = (blk->flags & AV1R_BLK_HAS_CHROMA) != 0;
    int bw = av1r_num4x4w[blk->mi_size] * 4, bh = av1r_num4x4h[blk->mi_size] * 4;
    int isII = isInter && mi_at(c, blk->mi_row, blk->mi_col)->ref_frame[1] == AV1R_INTRA_FRAME;
    for (int plane = 0; plane < 1 + hasChroma * 2; plane++) {
        int psz = plane_size(blk->mi_size, plane);
        int n4w = av1r_num4x4w[psz], n4h = av1r_num4x4h[psz];
        int log2W = 2 + av1r_miw_log2[psz], log2H = 2 + av1r_mih_log2[psz];
        int subX = plane ? hd->subx : 0, subY = plane ? hd->suby : 0;
        int baseX = (blk->mi_col >> subX) * 4, baseY = (blk->mi_row >> subY) * 4;
        int candRow = (blk->mi_row >> subY) << subY, candCol = (blk->mi_col >> subX) << subX;
        if (isII) {
            int im = blk->interintra_mode;
            int mode = im == AV1R_II_DC_PRED ? AV1R_DC_PRED : im == AV1R_II_V_PRED ? AV1R_V_PRED
                : im == AV1R_II_H_PRED ? AV1R_H_PRED : AV1R_SMOOTH_PRED;
            static _Thread_local uint8_t pred[64 * 64];
            IntraArgs a = {plane, baseX, baseY, log2W, log2H, blk};
            int haveL = plane == 0 ? (blk->flags & AV1R_BLK_AVAIL_L) != 0 : (blk->flags & AV1R_BLK_AVAIL_L_UV) != 0;
            int haveA = plane == 0 ? (blk->flags & AV1R_BLK_AVAIL_U) != 0 : (blk->flags & AV1R_BLK_AVAIL_U_UV) != 0;
            predict_intra(c, &a, haveL, haveA, (blk->ii_edge >> (2 * plane)) & 1, (blk->ii_edge >> (2 * plane + 1)) & 1, mode, pred);
            for (int r = 0; r < (1 << log2H); r++)
                for (int cc = 0; cc < (1 << log2W); cc++)
                    PIX(c->cur, plane, baseX + cc, baseY + r) = pred[r * 64 + cc];
        }
        if (isInter) {
            int predW = bw >> subX, predH = bh >> subY;
            int someUseIntra = 0;
            for (int r = 0; r < (n4h << subY); r++)
                for (int cc = 0; cc < (n4w << subX); cc++)
                    if (mi_at(c, candRow + r, candCol + cc)->ref_frame[0] == AV1R_INTRA_FRAME)
                        someUseIntra = 1;
            if (someUseIntra) {
                predW = n4w * 4;
                predH = n4h * 4;
                candRow = blk->mi_row;
                candCol = blk->mi_col;
            }
            int r = 0;
            for (int y = 0; y < n4h * 4; y += predH) {
                int cc = 0;
                for (int x = 0; x < n4w * 4; x += predW) {
                    predict_inter(c, blk, plane, baseX + x, baseY + y, predW, predH, candRow + r, candCol + cc);
                    cc++;
                }
                r++;
            }
        }
    }
}

/* ======================================================================================
 * Loop filter (decoder/LoopFilter.cpp)
 * ==================================================================================== */
typedef struct LfCtx {
    oracle_ctx* c;
    OFrame* f;
} LfCtx;

static int lf_limit(int sharp, int lvl)
{
    int shift = sharp > 4 ? 2 : (sharp > 0 ? 1 : 0);
    return sharp > 0 ? CLIP3(1, 9 - sharp, lvl >> shift) : MAX(1, lvl >> shift);
}
/* getFilterStrength / getLvl / getDeltaLF (LoopFilter.cpp:301-359) */
static void lf_strength(const oracle_ctx* c, int row, int col, int plane, int pass, int* lvl, int* limit, int* blimit, int* thresh)
{
    const av1r_frame_hdr* h = c->h;
    const av1r_mi* info = mi_at(c, row, col);
    int ref = info->ref_frame[0];
    int mode = info->y_mode;
    int modeType = mode >= AV1R_NEARESTMV && mode != AV1R_GLOBALMV && mode != AV1R_GLOBAL_GLOBALMV;
    int deltaLF = h->delta_lf_multi ? info->delta_lf[plane == 0 ? pass : plane + 1] : info->delta_lf[0];
    int i = plane == 0 ? pass : plane + 1;
    /* lvlSeg is an int8_t in the reference (LoopFilter.cpp:329-349) */
    int8_t l = (int8_t)CLIP3(0, 63, deltaLF + h->lf_level[i]);
    if (h->lf_delta_enabled) {
        int nShift = l >> 5;
        if (ref == AV1R_INTRA_FRAME)
            l = (int8_t)(l + (h->lf_ref_deltas[AV1R_INTRA_FRAME] << nShift));
        else
            l = (int8_t)(l + (h->lf_ref_deltas[ref & 7] << nShift) + (h->lf_mode_deltas[modeType] << nShift));
        l = (int8_t)CLIP3(0, 63, l);
    }
    *lvl = l;
    *limit = lf_limit(h->lf_sharpness, l);
    *blimit = 2 * (l + 2) + *limit;
    *thresh = l >> 4;
}

/* sampleFilter + getFilterMask + narrowFilter + wideFilter (LoopFilter.cpp:127-289) */
static void lf_sample(OFrame* f, int x, int y, int plane, int limit, int blimit, int thresh, int dx, int dy, int filterSize)
{
#define P(k) PIX(f, plane, x - dx * ((k) + 1), y - dy * ((k) + 1))
#define Q(k) PIX(f, plane, x + dx * (k), y + dy * (k))
    int q0 = Q(0), q1 = Q(1), q2 = Q(2), q3 = Q(3);
    int p0 = P(0), p1 = P(1), p2 = P(2), p3 = P(3);
    int q4 = 0, q5 = 0, q6 = 0, p4 = 0, p5 = 0, p6 = 0;
    if (filterSize == 16) {
        q4 = Q(4); q5 = Q(5); q6 = Q(6);
        p4 = P(4); p5 = P(5); p6 = P(6);
    }
    int hev = (iabs(p1 - p0) > thresh) | (iabs(q1 - q0) > thresh);
    int filterLen = filterSize == 4 ? 4 : (plane ? 6 : (filterSize == 8 ? 8 : 16));
    int mask = 0;
    mask |= iabs(p1 - p0) > limit;
    mask |= iabs(q1 - q0) > limit;
    mask |= iabs(p0 - q0) * 2 + iabs(p1 - q1) / 2 > blimit;
    if (filterLen >= 6) {
        mask |= iabs(p2 - p1) > limit;
        mask |= iabs(q2 - q1) > limit;
    }
    if (filterLen >= 8) {
        mask |= iabs(p3 - p2) > limit;
        mask |= iabs(q3 - q2) > limit;
    }
    if (mask)
        return;
    int flat = 0, flat2 = 0;
    if (filterSize >= 8) {
        int m = (iabs(p1 - p0) > 1) | (iabs(q1 - q0) > 1) | (iabs(p2 - p0) > 1) | (iabs(q2 - q0) > 1);
        if (filterLen >= 8)
            m |= (iabs(p3 - p0) > 1) | (iabs(q3 - q0) > 1);
        flat = !m;
    }
    if (filterSize >= 16) {
        int m = (iabs(p6 - p0) > 1) | (iabs(q6 - q0) > 1) | (iabs(p5 - p0) > 1) | (iabs(q5 - q0) > 1)
            | (iabs(p4 - p0) > 1) | (iabs(q4 - q0) > 1);
        flat2 = !m;
    }
    if (filterSize == 4 || !flat) {
        /* narrowFilter (LoopFilter.cpp:145-173) */
        int ps0 = p0 - 128, ps1 = p1 - 128, qs0 = q0 - 128, qs1 = q1 - 128;
        int filter = hev ? CLIP3(-128, 127, ps1 - qs1) : 0;
        filter = CLIP3(-128, 127, filter + 3 * (qs0 - ps0));
        int filter1 = CLIP3(-128, 127, filter + 4) >> 3;
        int filter2 = CLIP3(-128, 127, filter + 3) >> 3;
        Q(0) = (uint8_t)(CLIP3(-128, 127, qs0 - filter1) + 128);
        P(0) = (uint8_t)(CLIP3(-128, 127, ps0 + filter2) + 128);
        if (!hev) {
            filter = r2(filter1, 1);
            Q(1) = (uint8_t)(CLIP3(-128, 127, qs1 - filter) + 128);
            P(1) = (uint8_t)(CLIP3(-128, 127, ps1 + filter) + 128);
        }
    } else {
        /* wideFilter (LoopFilter.cpp:174-205) */
        int log2Size = (filterSize == 8 || !flat2) ? 3 : 4;
        int n = log2Size == 4 ? 6 : (!plane ? 3 : 2);
        int n2 = (log2Size == 3 && !plane) ? 0 : 1;
        int F[12];
        for (int i = -n; i < n; i++) {
            int t = 0;
            for (int j = -n; j <= n; j++) {
                int p = CLIP3(-(n + 1), n, i + j);
                int tap = (iabs(j) <= n2) ? 2 : 1;
                t += PIX(f, plane, x + p * dx, y + p * dy) * tap;
            }
            F[i + n] = r2(t, log2Size);
        }
        for (int i = -n; i < n; i++)
            PIX(f, plane, x + i * dx, y + i * dy) = (uint8_t)F[i + n];
    }
#undef P
#undef Q
}

/* LoopFilter::filter + loop_filter_edge (LoopFilter.cpp:40-126) */
static void loop_filter(oracle_ctx* c, OFrame* f)
{
    const av1r_frame_hdr* h = c->h;
    if (!h->lf_level[0] && !h->lf_level[1])
        return;
    for (int plane = 0; plane < 3; plane++) {
        if (!(plane == 0 || h->lf_level[1 + plane]))
            continue;
        int subX = plane ? h->subx : 0, subY = plane ? h->suby : 0;
        for (int pass = 0; pass < 2; pass++) {
            int rowStep = plane == 0 ? 1 : (1 << h->suby), colStep = plane == 0 ? 1 : (1 << h->subx);
            int dx = pass == 0, dy = pass == 1;
            for (int row0 = 0; row0 < h->mi_rows; row0 += rowStep)
                for (int col0 = 0; col0 < h->mi_cols; col0 += colStep) {
                    int x = col0 * 4, y = row0 * 4;
                    int row = row0 | subY, col = col0 | subX;
                    /* isOnScreen (LoopFilter.cpp:361-370) */
                    if (x >= h->frame_width || y >= h->frame_height) continue;
                    if (!pass && !x) continue;
                    if (pass && !y) continue;
                    int xP = x >> subX, yP = y >> subY;
                    int prevRow = row - (dy << subY), prevCol = col - (dx << subX);
                    const av1r_mi* info = mi_at(c, row, col);
                    int txSz = info->lf_tx[plane];
                    int psz = plane_size(info->mi_size, plane);
                    int skip = info->flags & AV1R_MI_SKIP;
                    int isIntra = info->ref_frame[0] <= AV1R_INTRA_FRAME;
                    int prevTx = mi_at(c, prevRow, prevCol)->lf_tx[plane];
                    int isBlockEdge = !pass ? !(xP % (av1r_num4x4w[psz] * 4)) : !(yP % (av1r_num4x4h[psz] * 4));
                    int isTxEdge = !pass ? !(xP % av1r_tx_w[txSz]) : !(yP % av1r_tx_h[txSz]);
                    int apply = isTxEdge && (isBlockEdge || !skip || isIntra);
                    int base = !pass ? MIN(av1r_tx_w[prevTx], av1r_tx_w[txSz]) : MIN(av1r_tx_h[prevTx], av1r_tx_h[txSz]);
                    int filterSize = !plane ? MIN(16, base) : MIN(8, base);
                    int lvl, limit, blimit, thresh;
                    lf_strength(c, row, col, plane, pass, &lvl, &limit, &blimit, &thresh);
                    if (!lvl)
                        lf_strength(c, prevRow, prevCol, plane, pass, &lvl, &limit, &blimit, &thresh);
                    if (!(apply && lvl > 0))
                        continue;
                    for (int i = 0; i < 4; i++)
                        lf_sample(f, xP + dy * i, yP + dx * i, plane, limit, blimit, thresh, dx, dy, filterSize);
                }
        }
    }
}

/* ======================================================================================
 * CDEF (decoder/Cdef.cpp)
 * ==================================================================================== */
static int constrain(int diff, int threshold, int damping)
{
    if (!threshold) return 0;
    int adj = MAX(0, damping - floor_log2(threshold));
    int sign = diff < 0 ? -1 : 1;
    return sign * CLIP3(0, iabs(diff), threshold - (iabs(diff) >> adj));
}
/* cdefDirection (Cdef.cpp:203-261) */
static void cdef_direction(const OFrame* f, int r, int col, int* yDir, int* var)
{
    int cost[8] = {0}, partial[8][15];
    memset(partial, 0, sizeof(partial));
    int x0 = col << 2, y0 = r << 2;
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            int x = PIX(f, 0, x0 + j, y0 + i) - 128;
            partial[0][i + j] += x;
            partial[1][i + j / 2] += x;
            partial[2][i] += x;
            partial[3][3 + i - j / 2] += x;
            partial[4][7 + i - j] += x;
            partial[5][3 - i / 2 + j] += x;
            partial[6][j] += x;
            partial[7][i / 2 + j] += x;
        }
    for (int i = 0; i < 8; i++) {
        cost[2] += partial[2][i] * partial[2][i];
        cost[6] += partial[6][i] * partial[6][i];
    }
    cost[2] *= av1r_cdef_div_table[8];
    cost[6] *= av1r_cdef_div_table[8];
    for (int i = 0; i < 7; i++) {
        cost[0] += (partial[0][i] * partial[0][i] + partial[0][14 - i] * partial[0][14 - i]) * av1r_cdef_div_table[i + 1];
        cost[4] += (partial[4][i] * partial[4][i] + partial[4][14 - i] * partial[4][14 - i]) * av1r_cdef_div_table[i + 1];
    }
    cost[0] += partial[0][7] * partial[0][7] * av1r_cdef_div_table[8];
    cost[4] += partial[4][7] * partial[4][7] * av1r_cdef_div_table[8];
    for (int i = 1; i < 8; i += 2) {
        for (int j = 0; j < 5; j++) cost[i] += partial[i][3 + j] * partial[i][3 + j];
        cost[i] *= av1r_cdef_div_table[8];
        for (int j = 0; j < 3; j++)
            cost[i] += (partial[i][j] * partial[i][j] + partial[i][10 - j] * partial[i][10 - j]) * av1r_cdef_div_table[2 * j + 2];
    }
    int best = 0;
    *yDir = 0;
    for (int i = 0; i < 8; i++)
        if (cost[i] > best) {
            best = cost[i];
            *yDir = i;
        }
    *var = (best - cost[(*yDir + 4) & 7]) >> 10;
}
/* cdefFilter + cdef_get_at (Cdef.cpp:140-198) */
static void cdef_filter(const oracle_ctx* c, OFrame* out, const OFrame* in, int plane, int r, int col, int priStr, int secStr, int damping, int dir)
{
    const av1r_frame_hdr* h = c->h;
    int subX = plane ? h->subx : 0, subY = plane ? h->suby : 0;
    int x0 = (col * 4) >> subX, y0 = (r * 4) >> subY;
    int w = 8 >> subX, hh = 8 >> subY;
    for (int i = 0; i < hh; i++)
        for (int j = 0; j < w; j++) {
            int sum = 0;
            int x = PIX(in, plane, x0 + j, y0 + i);
            int mx = x, mn = x;
            for (int k = 0; k < 2; k++)
                for (int sign = -1; sign <= 1; sign += 2) {
                    for (int s = 0; s < 3; s++) {
                        int d = s == 0 ? dir : ((dir + (s == 1 ? -2 : 2)) & 7);
                        int yy = y0 + i + sign * av1r_cdef_directions[d][k][0];
                        int xx = x0 + j + sign * av1r_cdef_directions[d][k][1];
                        int cr = (yy << subY) >> 2, cc = (xx << subX) >> 2;
                        if (!(cc >= 0 && cc < h->mi_cols && cr >= 0 && cr < h->mi_rows))
                            continue;
                        int p = PIX(in, plane, xx, yy);
                        if (s == 0)
                            sum += av1r_cdef_pri_taps[priStr & 1][k] * constrain(p - x, priStr, damping);
                        else
                            sum += av1r_cdef_sec_taps[priStr & 1][k] * constrain(p - x, secStr, damping);
                        mx = MAX(p, mx);
                        mn = MIN(p, mn);
                    }
                }
            PIX(out, plane, x0 + j, y0 + i) = (uint8_t)CLIP3(mn, mx, x + ((8 + sum - (sum < 0)) >> 4));
        }
}
/* Cdef::filter + cdef_block (Cdef.cpp:41-101) */
static OFrame* cdef(oracle_ctx* c, OFrame* in)
{
    const av1r_frame_hdr* h = c->h;
    OFrame* out = frame_copy(in);
    for (int r = 0; r < h->mi_rows; r += 2)
        for (int col = 0; col < h->mi_cols; col += 2) {
            int idx = c->b->cdef_idx[(r >> 4) * h->cdef_cols + (col >> 4)];
            if (idx == -1) continue;
            int skip = (mi_at(c, r, col)->flags & AV1R_MI_SKIP) && (mi_at(c, r + 1, col)->flags & AV1R_MI_SKIP)
                && (mi_at(c, r, col + 1)->flags & AV1R_MI_SKIP) && (mi_at(c, r + 1, col + 1)->flags & AV1R_MI_SKIP);
            if (skip) continue;
            int yDir, var;
            cdef_direction(in, r, col, &yDir, &var);
            int priStr = h->cdef_y_pri[idx], secStr = h->cdef_y_sec[idx];
            int dir = priStr == 0 ? 0 : yDir;
            int varStr = (var >> 6) ? MIN(floor_log2(var >> 6), 12) : 0;
            priStr = var ? (priStr * (4 + varStr) + 8) >> 4 : 0;
            int damping = h->cdef_damping;
            cdef_filter(c, out, in, 0, r, col, priStr, secStr, damping, dir);
            priStr = h->cdef_uv_pri[idx];
            secStr = h->cdef_uv_sec[idx];
            dir = priStr == 0 ? 0 : av1r_cdef_uv_dir420[yDir];
            damping = h->cdef_damping - 1;
            cdef_filter(c, out, in, 1, r, col, priStr, secStr, damping, dir);
            cdef_filter(c, out, in, 2, r, col, priStr, secStr, damping, dir);
        }
    return out;
}

/* ======================================================================================
 * Loop restoration (decoder/LoopRestoration.cpp)
 * ==================================================================================== */
typedef struct Stripe {
    int start, end;
} Stripe;
typedef struct LrCtx {
    const OFrame* cdefF;
    const OFrame* curF;
    OFrame* out;
    int plane;
    Stripe st;
} LrCtx;

/* get_source_sample (LoopRestoration.cpp:234-246) */
/* the widest unit: the last one of a row spans up to 1.5 unit sizes - 1 (count_units_in_frame
 * rounds, LoopRestoration.cpp:32-35), i.e. 383 px at 256 */
#define LR_MAXW 384
static inline int lr_src(const LrCtx* L, int x, int y)
{
    if (y < L->st.start) {
        y = MAX(L->st.start - 2, y);
        return PIX(L->curF, L->plane, x, y);
    } else if (y >= L->st.end) {
        y = MIN(L->st.end + 1, y);
        return PIX(L->curF, L->plane, x, y);
    }
    return PIX(L->cdefF, L->plane, x, y);
}
/* wienerFilter (LoopRestoration.cpp:247-277) */
static void lr_wiener(const LrCtx* L, const av1r_lr_unit* u, int x, int y, int w, int h)
{
    int vf[7], hf[7];
    for (int pass = 0; pass < 2; pass++) {
        int* f = pass ? hf : vf;
        f[3] = 128;
        for (int i = 0; i < 3; i++) {
            int cc = u->wiener[pass][i];
            f[i] = cc;
            f[6 - i] = cc;
            f[3] -= 2 * cc;
        }
    }
    const int R0 = 3, R1 = 11;
    int offset = 1 << (8 + 7 - R0 - 1);
    int limit = (1 << (8 + 1 + 7 - R0)) - 1;
    static _Thread_local int inter[64 + 6][LR_MAXW];
    for (int r = 0; r < h + 6; r++)
        for (int cc = 0; cc < w; cc++) {
            int s = 0;
            for (int t = 0; t < 7; t++)
                s += hf[t] * lr_src(L, x + cc + t - 3, y + r - 3);
            int v = r2(s, R0);
            inter[r][cc] = CLIP3(-offset, limit - offset, v);
        }
    for (int r = 0; r < h; r++)
        for (int cc = 0; cc < w; cc++) {
            int s = 0;
            for (int t = 0; t < 7; t++)
                s += vf[t] * inter[r + t][cc];
            PIX(L->out, L->plane, x + cc, y + r) = (uint8_t)CLIP1(r2(s, R1));
        }
}
/* boxFilter with boxsum1/boxsum2 (LoopRestoration.cpp:284-430); the box sums are
 * evaluated directly (the reference's own #if 0 branch asserts they are equal). */
static void lr_box(const LrCtx* L, int x, int y, int w, int h, int set, int pass, int r, int* F /* [h][w] stride LR_MAXW */)
{
    static _Thread_local int A[66][LR_MAXW + 2], Bv[66][LR_MAXW + 2];
    int eps = av1r_sgr_params[set][pass * 2 + 1];
    int n = (2 * r + 1) * (2 * r + 1);
    int n2e = n * n * eps;
    int s = ((1 << 20) + n2e / 2) / n2e;
    int oneOverN = ((1 << 12) + (n / 2)) / n;
    for (int i = -1; i < h + 1; i++)
        for (int j = -1; j < w + 1; j++) {
            int a = 0, b = 0;
            for (int dy = -r; dy <= r; dy++)
                for (int dx = -r; dx <= r; dx++) {
                    int cv = lr_src(L, x + j + dx, y + i + dy);
                    a += cv * cv;
                    b += cv;
                }
            int p = MAX(0, a * n - b * b);
            /* 32-bit int arithmetic as in the reference (LoopRestoration.cpp:380-381) */
            int z = (int)((uint32_t)p * (uint32_t)s + (1u << 19)) >> 20;
            int a2;
            if (z >= 255) a2 = 256;
            else if (z == 0) a2 = 1;
            else a2 = ((z << 8) + (z / 2)) / (z + 1);
            int b2 = ((1 << 8) - a2) * b * oneOverN;
            A[i + 1][j + 1] = a2;
            Bv[i + 1][j + 1] = r2(b2, 12);
        }
    for (int i = 0; i < h; i++) {
        int shift = (pass == 0 && (i & 1)) ? 4 : 5;
        for (int j = 0; j < w; j++) {
            int a = 0, b = 0;
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    int wt;
                    if (pass == 0) wt = ((i + dy) & 1) ? (dx == 0 ? 6 : 5) : 0;
                    else wt = (dx == 0 || dy == 0) ? 4 : 3;
                    a += wt * A[i + dy + 1][j + dx + 1];
                    b += wt * Bv[i + dy + 1][j + dx + 1];
                }
            int v = a * PIX(L->cdefF, L->plane, x + j, y + i) + b;
            F[i * LR_MAXW + j] = r2(v, 8 + shift - 4);
        }
    }
}
/* selfGuidedFilter (LoopRestoration.cpp:444-479) */
static void lr_sgr(const LrCtx* L, const av1r_lr_unit* u, int x, int y, int w, int h)
{
    static _Thread_local int flt0[64 * LR_MAXW], flt1[64 * LR_MAXW];
    int set = u->sgr_set;
    int r0 = av1r_sgr_params[set][0], r1 = av1r_sgr_params[set][2];
    if (r0) lr_box(L, x, y, w, h, set, 0, r0, flt0);
    if (r1 && r0 != r1) lr_box(L, x, y, w, h, set, 1, r1, flt1);
    int w0 = u->sgr_xqd[0], w1 = u->sgr_xqd[1], w2 = (1 << 7) - w0 - w1;
    for (int i = 0; i < h; i++)
        for (int j = 0; j < w; j++) {
            int uu = PIX(L->cdefF, L->plane, x + j, y + i) << 4;
            int v = w1 * uu;
            v += r0 ? w0 * flt0[i * LR_MAXW + j] : w0 * uu;
            v += r1 ? w2 * flt1[i * LR_MAXW + j] : w2 * uu;
            int s = r2(v, 4 + 7);
            PIX(L->out, L->plane, x + j, y + i) = (uint8_t)CLIP1(s);
        }
}
/* LoopRestoration::filter + forEachPlane/Unit/Stripe/Block (LoopRestoration.cpp:33-219) */
static OFrame* loop_restoration(oracle_ctx* c, OFrame* cdefF, OFrame* curF)
{
    const av1r_frame_hdr* h = c->h;
    if (!h->uses_lr) {
        frame_ref(cdefF);
        return cdefF;
    }
    frame_extend_border(cdefF, 3);
    frame_extend_border(curF, 3);
    OFrame* out = frame_copy(cdefF);
    for (int p = 0; p < 3; p++) {
        if (h->lr_type[p] == AV1R_RESTORE_NONE) continue;
        int subX = p ? h->subx : 0, subY = p ? h->suby : 0;
        int unitSize = h->lr_unit_size[p];
        int rows = h->lr_unit_rows[p], cols = h->lr_unit_cols[p];
        int planeEndX = r2(h->frame_width, subX), planeEndY = r2(h->frame_height, subY);
        for (int ur = 0; ur < rows; ur++)
            for (int uc = 0; uc < cols; uc++) {
                const av1r_lr_unit* u = &c->b->lr_units[h->lr_unit_off[p] + ur * cols + uc];
                if (u->type == AV1R_RESTORE_NONE) continue;
                /* UnitInfo (LoopRestoration.cpp:78-104) */
                int ux = uc * unitSize, uy = ur * unitSize;
                if (uy) uy -= 8 >> subY;
                int uw = (uc == cols - 1) ? planeEndX - ux : unitSize;
                int uh;
                if (ur == rows - 1) {
                    uh = planeEndY - uy;
                } else {
                    uh = unitSize;
                    if (!uy) uh -= 8 >> subY;
                }
                /* StripeInfo (LoopRestoration.cpp:106-135) */
                LrCtx L = {cdefF, curF, out, p, {0, 0}};
                int lumaY = uy << subY;
                int stripeNum = (lumaY + 8) / 64;
                L.st.start = (-8 + stripeNum * 64) >> subY;
                L.st.end = L.st.start + (64 >> subY);
                int unitEnd = uy + uh;
                for (;;) {
                    int yy = MAX(L.st.start, uy);
                    int hgt = MIN(L.st.end, uy + uh) - yy;
                    if (u->type == AV1R_RESTORE_WIENER) lr_wiener(&L, u, ux, yy, uw, hgt);
                    else if (u->type == AV1R_RESTORE_SGRPROJ) lr_sgr(&L, u, ux, yy, uw, hgt);
                    if (L.st.end >= unitEnd) break;
                    L.st.start = L.st.end;
                    L.st.end += 64 >> subY;
                }
            }
    }
    return out;
}

/* ======================================================================================
 * Frame driver: Decoder::decodeFrame + decode_frame_wrapup (Av1Decoder.cpp:128-192)
 * ==================================================================================== */
static void push_output(oracle_ctx* c, OFrame* f)
{
    if (c->nout == c->capout) {
        c->capout = c->capout ? c->capout * 2 : 16;
        c->outq = (OFrame**)realloc(c->outq, sizeof(OFrame*) * c->capout);
    }
    frame_ref(f);
    c->outq[c->nout++] = f;
}
static void update_store(oracle_ctx* c, int refresh, OFrame* f)
{
    for (int i = 0; i < 8; i++)
        if (refresh & (1 << i)) {
            frame_ref(f);
            frame_unref(c->store[i]);
            c->store[i] = f;
        }
}
static void set_stage(oracle_ctx* c, int s, OFrame* f)
{
    frame_unref(c->stage[s]);
    c->stage[s] = f;
}

oracle_ctx* oracle_create(void)
{
    oracle_ctx* c = (oracle_ctx*)calloc(1, sizeof(oracle_ctx));
    c->keep_stages = 1;
    return c;
}
void oracle_destroy(oracle_ctx* c)
{
    if (!c) return;
    for (int i = 0; i < 8; i++) frame_unref(c->store[i]);
    for (int i = c->headout; i < c->nout; i++) frame_unref(c->outq[i]);
    for (int i = 0; i < 4; i++) frame_unref(c->stage[i]);
    free(c->outq);
    free(c);
}
void oracle_set_keep_stages(oracle_ctx* c, int keep) { c->keep_stages = keep; }

int oracle_show_existing(oracle_ctx* c, int slot, int refresh)
{
    OFrame* f = c->store[slot];
    if (!f) return AV1R_E_INVALID;
    push_output(c, f);
    frame_ref(f);
    update_store(c, refresh, f);
    frame_unref(f);
    return AV1R_OK;
}

int oracle_decode_frame(oracle_ctx* c, const av1r_frame_batch* b)
{
    const av1r_frame_hdr* h = b->hdr;
    if (!h || h->version != AV1R_VERSION) return AV1R_E_INVALID;
    if (h->show_existing_frame) return oracle_show_existing(c, h->frame_to_show, h->refresh_frame_flags);
    if (h->bitdepth != 8 || h->subx != 1 || h->suby != 1) return AV1R_E_UNSUPPORTED;
    c->b = b;
    c->h = h;
    c->cur = frame_create(h->frame_width, h->frame_height);
    for (uint32_t i = 0; i < b->n_blocks; i++) {
        const av1r_block* blk = &b->blocks[i];
        compute_prediction(c, blk);
        if (!(getenv("ORACLE_NO_TB") && h->frame_type))
            for (uint32_t t = 0; t < blk->n_tbs; t++)
                decode_tb(c, &b->tbs[blk->first_tb + t]);
    }
    if (c->keep_stages) set_stage(c, AV1R_STAGE_RECON, frame_copy(c->cur));
    loop_filter(c, c->cur);
    if (c->keep_stages) set_stage(c, AV1R_STAGE_LF, frame_copy(c->cur));
    OFrame* cd = cdef(c, c->cur);
    if (c->keep_stages) { frame_ref(cd); set_stage(c, AV1R_STAGE_CDEF, cd); }
    OFrame* lr = loop_restoration(c, cd, c->cur);
    if (c->keep_stages) { frame_ref(lr); set_stage(c, AV1R_STAGE_LR, lr); }
    if (h->show_frame) push_output(c, lr);
    update_store(c, h->refresh_frame_flags, lr);
    frame_unref(lr);
    frame_unref(cd);
    frame_unref(c->cur);
    c->cur = NULL;
    c->b = NULL;
    c->h = NULL;
    return AV1R_OK;
}

int oracle_output_pending(oracle_ctx* c) { return c->nout - c->headout; }

static void copy_planes(const OFrame* f, uint8_t* y, int ys, uint8_t* u, int us, uint8_t* v, int vs)
{
    uint8_t* dst[3] = {y, u, v};
    int ds[3] = {ys, us, vs};
    for (int p = 0; p < 3; p++) {
        int w = p ? f->width >> 1 : f->width, hh = p ? f->height >> 1 : f->height;
        for (int r = 0; r < hh; r++)
            memcpy(dst[p] + (size_t)r * ds[p], f->data[p] + r * f->stride[p], w);
    }
}
int oracle_get_output(oracle_ctx* c, uint8_t* y, int ys, uint8_t* u, int us, uint8_t* v, int vs, int* width, int* height)
{
    if (c->headout == c->nout) return AV1R_E_NO_OUTPUT;
    OFrame* f = c->outq[c->headout];
    if (width) *width = f->width;
    if (height) *height = f->height;
    if (y) {
        copy_planes(f, y, ys, u, us, v, vs);
        c->headout++;
        frame_unref(f);
        if (c->headout == c->nout) c->headout = c->nout = 0;
    }
    return AV1R_OK;
}
int oracle_read_stage(oracle_ctx* c, int stage, int plane, uint8_t* dst, int ds)
{
    if (stage < 0 || stage > 3 || !c->stage[stage]) return AV1R_E_INVALID;
    const OFrame* f = c->stage[stage];
    int w = plane ? f->width >> 1 : f->width, hh = plane ? f->height >> 1 : f->height;
    for (int r = 0; r < hh; r++)
        memcpy(dst + (size_t)r * ds, f->data[plane] + r * f->stride[plane], w);
    return AV1R_OK;
}
