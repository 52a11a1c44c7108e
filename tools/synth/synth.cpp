// synth.cpp -- seeded synthetic AV1 frame-batch generator (bench / test input).
//
// No AV1 encoder exists in this image and no 1080p/4K stream exists in the reference's
// bits/ (SURVEY.md K9, 8d), so the bench workload (BASELINE.json configs[2]/[3]) is
// synthesised directly at the boundary: a seeded stream of av1r frame batches with the
// structure the reference's parser produces -- a partition tree per superblock, intra
// and inter blocks in decode order, transform blocks in Block::residual order
// (decoder/Block.cpp:262-301), intra edge-availability flags derived with the same
// per-superblock decoded-flag rules as BlockDecoded (decoder/Tile.cpp:42-75), mode-info
// grid, CDEF indices and loop-restoration units.  Distributions follow SURVEY.md 8d:
// 80 % inter blocks, 40 % of them compound (avg 50 / dist 20 / wedge 15 / diff 15),
// OBMC 10 %, local warp 5 %, MVs uniform +-64 px with 1/8-pel fractions, dual filters,
// eob buckets of the allintra histogram, LF 32/32/16/16, 8 CDEF strengths, Wiener on
// luma / self-guided on chroma.  Parity on these batches is oracle-vs-HIP.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "av1r.h"
#include "av1r_consts.h"

namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x1234567ull) {}
    uint32_t next()
    {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return (uint32_t)(s >> 16);
    }
    int uni(int lo, int hi) { return lo + (int)(next() % (uint32_t)(hi - lo + 1)); }
    bool p(int percent) { return (int)(next() % 100) < percent; }
};

const int kMaxTxRect[AV1R_BLOCK_SIZES] = {
    AV1R_TX_4X4, AV1R_TX_4X8, AV1R_TX_8X4, AV1R_TX_8X8, AV1R_TX_8X16, AV1R_TX_16X8, AV1R_TX_16X16,
    AV1R_TX_16X32, AV1R_TX_32X16, AV1R_TX_32X32, AV1R_TX_32X64, AV1R_TX_64X32, AV1R_TX_64X64,
    AV1R_TX_64X64, AV1R_TX_64X64, AV1R_TX_64X64, AV1R_TX_4X16, AV1R_TX_16X4, AV1R_TX_8X32,
    AV1R_TX_32X8, AV1R_TX_16X64, AV1R_TX_64X16};
const int kSplitTx[AV1R_TX_SIZES] = {
    AV1R_TX_4X4, AV1R_TX_4X4, AV1R_TX_8X8, AV1R_TX_16X16, AV1R_TX_32X32, AV1R_TX_4X4, AV1R_TX_4X4,
    AV1R_TX_8X8, AV1R_TX_8X8, AV1R_TX_16X16, AV1R_TX_16X16, AV1R_TX_32X32, AV1R_TX_32X32,
    AV1R_TX_4X8, AV1R_TX_8X4, AV1R_TX_8X16, AV1R_TX_16X8, AV1R_TX_16X32, AV1R_TX_32X16};

int bsize_of(int w, int h)
{
    for (int b = 0; b < AV1R_BLOCK_SIZES; b++)
        if (av1r_num4x4w[b] * 4 == w && av1r_num4x4h[b] * 4 == h) return b;
    return -1;
}
int txsize_of(int w, int h)
{
    for (int t = 0; t < AV1R_TX_SIZES; t++)
        if (av1r_tx_w[t] == w && av1r_tx_h[t] == h) return t;
    return -1;
}
// Block::get_tx_size for chroma (Block.cpp:205-220)
int uv_tx_size(int bs)
{
    int uvTx = kMaxTxRect[av1r_ss420[bs]];
    if (av1r_tx_w[uvTx] == 64 || av1r_tx_h[uvTx] == 64) {
        if (av1r_tx_w[uvTx] == 16) return AV1R_TX_16X32;
        if (av1r_tx_h[uvTx] == 16) return AV1R_TX_32X16;
        return AV1R_TX_32X32;
    }
    return uvTx;
}

int iabs(int v) { return v < 0 ? -v : v; }
int r2s(int x, int n) { return x >= 0 ? ((x + (1 << (n - 1))) >> n) : -((-x + (1 << (n - 1))) >> n); }
int64_t r2s64(int64_t x, int n)
{
    int64_t h = (int64_t)1 << (n - 1);
    return x >= 0 ? ((x + h) >> n) : -((-x + h) >> n);
}
// setupShear validity (Block.cpp:1179-1200) for generated local-warp parameters
bool shear_valid(const int32_t* wp)
{
    int alpha0 = std::max(-32768, std::min(32767, wp[2] - (1 << 16)));
    int beta0 = std::max(-32768, std::min(32767, wp[3]));
    int64_t d = wp[2];
    int n = 63 - __builtin_clzll((uint64_t)(d < 0 ? -d : d));
    int64_t e = (d < 0 ? -d : d) - ((int64_t)1 << n);
    int64_t f = n > 8 ? ((e + ((int64_t)1 << (n - 9))) >> (n - 8)) : (e << (8 - n));
    int divShift = n + 14;
    int divFactor = av1r_div_lut[f];
    int gamma0 = (int)std::max<int64_t>(-32768, std::min<int64_t>(32767, r2s64((int64_t)(wp[4] << 16) * divFactor, divShift)));
    int delta0 = (int)std::max<int64_t>(-32768, std::min<int64_t>(32767, wp[5] - r2s64((int64_t)(wp[3] * wp[4]) * divFactor, divShift) - (1 << 16)));
    int alpha = r2s(alpha0, 6) << 6, beta = r2s(beta0, 6) << 6, gamma = r2s(gamma0, 6) << 6, delta = r2s(delta0, 6) << 6;
    return (4 * iabs(alpha) + 7 * iabs(beta)) < (1 << 16) && (4 * iabs(gamma) + 4 * iabs(delta)) < (1 << 16);
}

struct Gen {
    int W, H, sb128, tiles_c, tiles_r;
    uint32_t seed;
    int frameNo = 0;
    int miCols, miRows, miStride, miRowsAlloc;
    std::vector<int> tileColStart, tileRowStart;  // mi units, with end sentinel
    av1r_frame_hdr hdr;
    std::vector<av1r_mi> mi;
    std::vector<av1r_block> blocks;
    std::vector<av1r_tb> tbs;
    std::vector<uint32_t> coefs;
    std::vector<int8_t> cdef;
    std::vector<av1r_lr_unit> lr;
    std::vector<uint8_t> rec;
    // BlockDecoded emulation (Tile.cpp:42-75): [plane][r+1][c+1]
    bool dec[3][34][34];
    int sbR, sbC;  // current SB origin (mi)
    int tileR0, tileR1, tileC0, tileC1;

    bool inside(int r, int c) const { return r >= tileR0 && r < tileR1 && c >= tileC0 && c < tileC1; }
    av1r_mi& M(int r, int c) { return mi[(size_t)r * miStride + c]; }

    void clear_flags(int r, int c)
    {
        int sb4 = sb128 ? 32 : 16;
        for (int p = 0; p < 3; p++) {
            int sub = p ? 1 : 0;
            int w4 = (tileC1 - c) >> sub, h4 = (tileR1 - r) >> sub;
            memset(dec[p], 0, sizeof(dec[p]));
            for (int y = -1; y <= (sb4 >> sub); y++)
                for (int x = -1; x <= (sb4 >> sub); x++) {
                    if (y < 0 && x < w4) dec[p][y + 1][x + 1] = true;
                    else if (x < 0 && y < h4) dec[p][y + 1][x + 1] = true;
                    else dec[p][y + 1][x + 1] = false;
                }
            dec[p][(sb4 >> sub) + 1][0] = false;
        }
    }
    bool flag(int p, int r, int c) const
    {
        if (r + 1 < 0 || c + 1 < 0 || r + 1 >= 34 || c + 1 >= 34) return false;
        return dec[p][r + 1][c + 1];
    }

    void setup_frame(Rng& rng)
    {
        memset(&hdr, 0, sizeof(hdr));
        hdr.version = AV1R_VERSION;
        hdr.frame_width = W;
        hdr.frame_height = H;
        hdr.mi_cols = miCols;
        hdr.mi_rows = miRows;
        hdr.mi_stride = miStride;
        hdr.mi_rows_alloc = miRowsAlloc;
        hdr.sb128 = sb128;
        hdr.subx = hdr.suby = 1;
        hdr.bitdepth = 8;
        hdr.show_frame = 1;
        bool key = frameNo == 0;
        hdr.frame_type = key ? 0 : 1;
        hdr.refresh_frame_flags = key ? 0xFF : (uint8_t)(1 << (frameNo % 7));
        hdr.enable_intra_edge_filter = 1;
        for (int i = 0; i < 8; i++) hdr.ref_frame_idx[i] = i < 7 ? i : -1;
        for (int r = 1; r < 8; r++) hdr.ref_dist[r] = key ? 0 : (uint8_t)(1 + (r * 3 + frameNo) % 6);
        for (int r = 0; r < 8; r++) {
            hdr.gm_params[r][2] = hdr.gm_params[r][5] = 1 << 16;
        }
        hdr.lf_level[0] = 32;
        hdr.lf_level[1] = 32;
        hdr.lf_level[2] = 16;
        hdr.lf_level[3] = 16;
        hdr.lf_delta_enabled = 1;
        const int8_t rd[8] = {1, 0, 0, 0, -1, 0, -1, -1};
        memcpy(hdr.lf_ref_deltas, rd, 8);
        hdr.cdef_damping = 5;
        hdr.cdef_bits = 3;
        for (int i = 0; i < 8; i++) {
            hdr.cdef_y_pri[i] = (uint8_t)rng.uni(0, 15);
            hdr.cdef_y_sec[i] = (uint8_t)(rng.uni(0, 3) == 3 ? 4 : rng.uni(0, 2));
            hdr.cdef_uv_pri[i] = (uint8_t)rng.uni(0, 15);
            hdr.cdef_uv_sec[i] = (uint8_t)(rng.uni(0, 3) == 3 ? 4 : rng.uni(0, 2));
        }
        hdr.cdef_rows = (miRows + 15) / 16;
        hdr.cdef_cols = (miCols + 15) / 16;
        mi.assign((size_t)miStride * miRowsAlloc, av1r_mi());
        for (auto& m : mi) {
            memset(&m, 0, sizeof(m));
            m.ref_frame[0] = 0;
            m.ref_frame[1] = -1;
        }
        blocks.clear();
        tbs.clear();
        coefs.clear();
    }

    void emit_coefs(Rng& rng, av1r_tb& t, bool skip)
    {
        t.coef_off = (uint32_t)coefs.size();
        t.coef_cnt = 0;
        if (skip) return;
        int tw = std::min<int>(av1r_tx_w[t.tx_size], 32), th = std::min<int>(av1r_tx_h[t.tx_size], 32);
        int area = tw * th;
        int b = rng.uni(0, 99), eob;
        if (b < 9) eob = 0;
        else if (b < 19) eob = rng.uni(1, 4);
        else if (b < 85) eob = rng.uni(5, 16);
        else if (b < 99) eob = rng.uni(17, 64);
        else eob = rng.uni(65, 256);
        eob = std::min(eob, area);
        // positions along anti-diagonals (the shape of the default zig-zag scan)
        int placed = 0;
        for (int d = 0; d < tw + th - 1 && placed < eob; d++)
            for (int i = 0; i <= d && placed < eob; i++) {
                int r = i, c = d - i;
                if (r >= th || c >= tw) continue;
                int lvl = 1;
                while (lvl < 12 && rng.p(50)) lvl++;
                if (placed == 0) lvl += rng.uni(0, 20);
                if (rng.p(50)) lvl = -lvl;
                if (placed > 0 && placed + 1 < eob && rng.p(30)) lvl = 0;  // interior zeros
                if (lvl) coefs.push_back(((uint32_t)lvl << 10) | (uint32_t)(r * tw + c));
                placed++;
            }
        t.coef_cnt = (uint16_t)(coefs.size() - t.coef_off);
        if (!t.coef_cnt) t.tx_type = AV1R_DCT_DCT;
    }

    int pick_tx_type(Rng& rng, int txSz)
    {
        int w = av1r_tx_w[txSz], h = av1r_tx_h[txSz];
        if (w == 64 || h == 64) return AV1R_DCT_DCT;
        if (w == 32 || h == 32) return rng.p(85) ? AV1R_DCT_DCT : AV1R_IDTX;
        return rng.p(50) ? AV1R_DCT_DCT : rng.uni(0, 15);
    }

    // TransformBlock records of one block in Block::residual order (Block.cpp:262-301)
    void emit_tbs(Rng& rng, uint32_t bi, int lumaTx, bool interBlk, bool skip)
    {
        av1r_block& B = blocks[bi];
        int bs = B.mi_size;
        int bw = av1r_num4x4w[bs] * 4, bh = av1r_num4x4h[bs] * 4;
        bool hasChroma = B.flags & AV1R_BLK_HAS_CHROMA;
        int wChunks = std::max(1, bw >> 6), hChunks = std::max(1, bh >> 6);
        int chunkBs = (wChunks > 1 || hChunks > 1) ? AV1R_BLOCK_64X64 : bs;
        int sbMask = sb128 ? 31 : 15;
        B.first_tb = (uint32_t)tbs.size();
        for (int cy = 0; cy < hChunks; cy++)
            for (int cx = 0; cx < wChunks; cx++)
                for (int p = 0; p < 1 + 2 * hasChroma; p++) {
                    int sub = p ? 1 : 0;
                    int txSz = p ? uv_tx_size(bs) : lumaTx;
                    int psz = p ? av1r_ss420[chunkBs] : chunkBs;
                    int cw = av1r_num4x4w[psz] * 4, ch = av1r_num4x4h[psz] * 4;
                    int baseX = (B.mi_col >> sub) * 4 + ((cx * 64) >> sub), baseY = (B.mi_row >> sub) * 4 + ((cy * 64) >> sub);
                    int blkX = (B.mi_col >> sub) * 4, blkY = (B.mi_row >> sub) * 4;
                    int tw = av1r_tx_w[txSz], th = av1r_tx_h[txSz];
                    for (int y = 0; y < ch; y += th)
                        for (int x = 0; x < cw; x += tw) {
                            av1r_tb t;
                            memset(&t, 0, sizeof(t));
                            t.block = bi;
                            t.plane = (uint8_t)p;
                            t.tx_size = (uint8_t)txSz;
                            t.x = (uint16_t)(baseX + x);
                            t.y = (uint16_t)(baseY + y);
                            t.tx_type = interBlk ? (uint8_t)pick_tx_type(rng, txSz) : (uint8_t)pick_tx_type(rng, txSz);
                            // edge flags exactly as TransformBlock::decode (TransformBlock.cpp:2379-2412)
                            int row = (t.y << sub) >> 2, col = (t.x << sub) >> 2;
                            int sr = (row & sbMask) >> sub, sc = (col & sbMask) >> sub;
                            int stepX = tw >> 2, stepY = th >> 2;
                            bool aL = p ? (B.flags & AV1R_BLK_AVAIL_L_UV) : (B.flags & AV1R_BLK_AVAIL_L);
                            bool aU = p ? (B.flags & AV1R_BLK_AVAIL_U_UV) : (B.flags & AV1R_BLK_AVAIL_U);
                            if (aL || t.x > blkX) t.flags |= AV1R_TB_HAVE_LEFT;
                            if (aU || t.y > blkY) t.flags |= AV1R_TB_HAVE_ABOVE;
                            if (flag(p, sr - 1, sc + stepX)) t.flags |= AV1R_TB_HAVE_AR;
                            if (flag(p, sr + stepY, sc - 1)) t.flags |= AV1R_TB_HAVE_BL;
                            emit_coefs(rng, t, skip);
                            tbs.push_back(t);
                            for (int i = 0; i < stepY; i++)
                                for (int j = 0; j < stepX; j++) {
                                    if (sr + i + 1 < 34 && sc + j + 1 < 34) dec[p][sr + i + 1][sc + j + 1] = true;
                                    for (int yy = 0; yy <= sub; yy++)
                                        for (int xx = 0; xx <= sub; xx++) {
                                            int rr = row + (i << sub) + yy, cc = col + (j << sub) + xx;
                                            if (rr < miRowsAlloc && cc < miStride) M(rr, cc).lf_tx[p] = (uint8_t)txSz;
                                        }
                                }
                        }
                }
        B.n_tbs = (uint32_t)tbs.size() - B.first_tb;
    }

    bool smooth_mode(int m) { return m == AV1R_SMOOTH_PRED || m == AV1R_SMOOTH_V_PRED || m == AV1R_SMOOTH_H_PRED; }

    void make_block(Rng& rng, int r, int c, int bs)
    {
        bool key = frameNo == 0;
        int bw4 = av1r_num4x4w[bs], bh4 = av1r_num4x4h[bs];
        av1r_block B;
        memset(&B, 0, sizeof(B));
        B.mi_row = (uint16_t)r;
        B.mi_col = (uint16_t)c;
        B.mi_size = (uint8_t)bs;
        B.qindex = 100;
        bool hasChroma = !((bh4 == 1 && (r & 1) == 0) || (bw4 == 1 && (c & 1) == 0));
        bool availU = inside(r - 1, c), availL = inside(r, c - 1);
        bool availUC = availU, availLC = availL;
        if (hasChroma) {
            if (bh4 == 1) availUC = inside(r - 2, c);
            if (bw4 == 1) availLC = inside(r, c - 2);
        } else {
            availUC = availLC = false;
        }
        uint32_t f = 0;
        if (hasChroma) f |= AV1R_BLK_HAS_CHROMA;
        if (availL) f |= AV1R_BLK_AVAIL_L;
        if (availU) f |= AV1R_BLK_AVAIL_U;
        if (availLC) f |= AV1R_BLK_AVAIL_L_UV;
        if (availUC) f |= AV1R_BLK_AVAIL_U_UV;
        bool inter = !key && rng.p(80);
        bool skip = rng.p(inter ? 30 : 5);
        if (skip) f |= AV1R_BLK_SKIP;
        int minWh = std::min(bw4, bh4) * 4;
        int ref0 = 0, ref1 = -1, ymode, uvmode = 0;
        int16_t mv[2][2] = {{0, 0}, {0, 0}};
        int filt = 0;
        int lumaTx = kMaxTxRect[bs];
        if (inter) {
            f |= AV1R_BLK_INTER;
            ref0 = rng.uni(1, 7);
            bool compound = minWh >= 8 && rng.p(40);
            for (int l = 0; l < 2; l++) {
                mv[l][0] = (int16_t)rng.uni(-512, 512);
                mv[l][1] = (int16_t)rng.uni(-512, 512);
            }
            filt = rng.uni(0, 2) | (rng.uni(0, 2) << 4);
            ymode = compound ? AV1R_NEW_NEWMV : AV1R_NEWMV;
            B.compound_type = AV1R_COMPOUND_AVERAGE;
            if (compound) {
                ref1 = rng.uni(1, 7);
                if (ref1 == ref0) ref1 = ref0 % 7 + 1;
                int ct = rng.uni(0, 99);
                if (ct < 50) B.compound_type = AV1R_COMPOUND_AVERAGE;
                else if (ct < 70) B.compound_type = AV1R_COMPOUND_DISTANCE;
                else if (ct < 85 && av1r_wedge_bits[bs]) {
                    B.compound_type = AV1R_COMPOUND_WEDGE;
                    B.wedge_index = (uint8_t)rng.uni(0, 15);
                    B.wedge_sign = (uint8_t)rng.uni(0, 1);
                } else {
                    B.compound_type = AV1R_COMPOUND_DIFFWTD;
                    B.mask_type = (uint8_t)rng.uni(0, 1);
                }
            } else if (bs >= AV1R_BLOCK_8X8 && bs <= AV1R_BLOCK_32X32 && rng.p(10)) {
                f |= AV1R_BLK_INTERINTRA;
                ref1 = 0;  // RefFrame[1] = INTRA_FRAME (Block.cpp:1244)
                B.interintra_mode = (uint8_t)rng.uni(0, 3);
                if (av1r_wedge_bits[bs] && rng.p(50)) {
                    f |= AV1R_BLK_WEDGE_II;
                    B.compound_type = AV1R_COMPOUND_WEDGE;
                    B.wedge_index = (uint8_t)rng.uni(0, 15);
                } else {
                    B.compound_type = AV1R_COMPOUND_INTRA;
                }
                int sbRow = r & (sb128 ? 31 : 15), sbCol = c & (sb128 ? 31 : 15);
                for (int p = 0; p < 1 + 2 * hasChroma; p++) {
                    int sub = p ? 1 : 0, psz = p ? av1r_ss420[bs] : bs;
                    if (flag(p, (sbRow >> sub) - 1, (sbCol >> sub) + av1r_num4x4w[psz])) B.ii_edge |= 1 << (2 * p);
                    if (flag(p, (sbRow >> sub) + av1r_num4x4h[psz], (sbCol >> sub) - 1)) B.ii_edge |= 2 << (2 * p);
                }
            } else if (minWh >= 8 && rng.p(15)) {
                int m = rng.uni(0, 2);
                if (m < 2) {
                    B.motion_mode = AV1R_OBMC_CAUSAL;
                } else {
                    B.motion_mode = AV1R_LOCALWARP;
                    int32_t wp[6];
                    wp[2] = (1 << 16) + rng.uni(-2000, 2000);
                    wp[3] = rng.uni(-1500, 1500);
                    wp[4] = rng.uni(-1500, 1500);
                    wp[5] = (1 << 16) + rng.uni(-2000, 2000);
                    wp[0] = mv[0][1] * (1 << 13) + rng.uni(-4096, 4096);
                    wp[1] = mv[0][0] * (1 << 13) + rng.uni(-4096, 4096);
                    memcpy(B.local_warp, wp, sizeof(wp));
                    if (shear_valid(wp)) f |= AV1R_BLK_LOCAL_VALID;
                }
            }
            if (!skip && rng.p(50) && lumaTx != AV1R_TX_4X4) lumaTx = kSplitTx[lumaTx];
        } else {
            ymode = rng.uni(0, 12);
            if (ymode >= AV1R_V_PRED && ymode <= AV1R_D67_PRED) B.angle_delta_y = (int8_t)rng.uni(-3, 3);
            bool cflOk = bw4 <= 8 && bh4 <= 8;
            uvmode = rng.uni(0, cflOk ? 13 : 12);
            if (uvmode >= AV1R_V_PRED && uvmode <= AV1R_D67_PRED) B.angle_delta_uv = (int8_t)rng.uni(-3, 3);
            B.cfl_alpha_u = (int8_t)rng.uni(-16, 16);
            B.cfl_alpha_v = (int8_t)rng.uni(-16, 16);
            if (ymode == AV1R_DC_PRED && bw4 <= 8 && bh4 <= 8 && rng.p(30)) {
                f |= AV1R_BLK_FILTER_INTRA;
                B.filter_intra_mode = (uint8_t)rng.uni(0, 4);
            }
            int d = rng.uni(0, 2);
            while (d-- > 0 && lumaTx != AV1R_TX_4X4) lumaTx = kSplitTx[lumaTx];
            if (f & AV1R_BLK_FILTER_INTRA) {
                while (av1r_tx_w[lumaTx] > 32 || av1r_tx_h[lumaTx] > 32) lumaTx = kSplitTx[lumaTx];
            }
            // intra edge smoothness (IntraPredict.cpp:211-254)
            if (availU && smooth_mode(M(r - 1, c).y_mode) && M(r - 1, c).ref_frame[0] <= 0) f |= AV1R_BLK_SMOOTH_A_Y;
            if (availL && smooth_mode(M(r, c - 1).y_mode) && M(r, c - 1).ref_frame[0] <= 0) f |= AV1R_BLK_SMOOTH_L_Y;
            if (availUC) {
                int rr = r - 1, cc = c;
                if (!(c & 1)) cc++;
                if (r & 1) rr--;
                const av1r_mi& m = M(rr, cc);
                if (m.ref_frame[0] <= 0 && smooth_mode(m.uv_mode)) f |= AV1R_BLK_SMOOTH_A_UV;
            }
            if (availLC) {
                int rr = r, cc = c - 1;
                if (c & 1) cc--;
                if (!(r & 1)) rr++;
                const av1r_mi& m = M(rr, cc);
                if (m.ref_frame[0] <= 0 && smooth_mode(m.uv_mode)) f |= AV1R_BLK_SMOOTH_L_UV;
            }
            B.max_luma_w = (uint16_t)(c * 4 + bw4 * 4);
            B.max_luma_h = (uint16_t)(r * 4 + bh4 * 4);
        }
        if (inter && (B.flags & AV1R_BLK_INTERINTRA)) ymode = AV1R_NEWMV;
        B.y_mode = (uint8_t)ymode;
        B.uv_mode = (uint8_t)(hasChroma && !inter ? uvmode : 0);  // as the parser: intra blocks only
        B.flags = f;
        // smooth-neighbour luma check of the reference reads YMode regardless of inter-ness
        if (!inter) {
            B.flags &= ~(AV1R_BLK_SMOOTH_A_Y | AV1R_BLK_SMOOTH_L_Y);
            if (availU && smooth_mode(M(r - 1, c).y_mode)) B.flags |= AV1R_BLK_SMOOTH_A_Y;
            if (availL && smooth_mode(M(r, c - 1).y_mode)) B.flags |= AV1R_BLK_SMOOTH_L_Y;
        }
        for (int y = 0; y < bh4; y++)
            for (int x = 0; x < bw4; x++) {
                av1r_mi& m = M(r + y, c + x);
                m.y_mode = (uint8_t)ymode;
                if (!inter && hasChroma) m.uv_mode = (uint8_t)uvmode;
                m.ref_frame[0] = (int8_t)ref0;
                m.ref_frame[1] = (int8_t)ref1;
                if (inter) {
                    m.filt = (uint8_t)filt;
                    memcpy(m.mv, mv, sizeof(mv));
                }
                m.mi_size = (uint8_t)bs;
                m.flags = (uint8_t)((skip ? AV1R_MI_SKIP : 0) | (inter ? AV1R_MI_INTER : 0));
            }
        {  // v2: the block's mode info (what it wrote over its units above)
            const av1r_mi& m = M(r, c);
            memcpy(B.mv, m.mv, sizeof(B.mv));
            B.ref_frame[0] = m.ref_frame[0];
            B.ref_frame[1] = m.ref_frame[1];
            B.filt = m.filt;
            memcpy(B.delta_lf, m.delta_lf, sizeof(B.delta_lf));
        }
        uint32_t bi = (uint32_t)blocks.size();
        blocks.push_back(B);
        emit_tbs(rng, bi, lumaTx, inter, skip);
    }

    void partition(Rng& rng, int r, int c, int size4)
    {
        if (r >= miRows || c >= miCols) return;
        bool crosses = r + size4 > miRows || c + size4 > miCols;
        int sizePx = size4 * 4;
        if (size4 > 2 && (crosses || (sizePx > 32 ? rng.p(85) : rng.p(sizePx == 32 ? 55 : 35)))) {
            int h = size4 / 2;
            partition(rng, r, c, h);
            partition(rng, r, c + h, h);
            partition(rng, r + h, c, h);
            partition(rng, r + h, c + h, h);
            return;
        }
        if (size4 == 2 && rng.p(25)) {  // PARTITION_SPLIT of an 8x8 into 4x4s, or 4x8/8x4 pairs
            int k = rng.uni(0, 2);
            if (k == 0) {
                make_block(rng, r, c, AV1R_BLOCK_4X4);
                make_block(rng, r, c + 1, AV1R_BLOCK_4X4);
                make_block(rng, r + 1, c, AV1R_BLOCK_4X4);
                make_block(rng, r + 1, c + 1, AV1R_BLOCK_4X4);
            } else if (k == 1) {
                make_block(rng, r, c, AV1R_BLOCK_8X4);
                make_block(rng, r + 1, c, AV1R_BLOCK_8X4);
            } else {
                make_block(rng, r, c, AV1R_BLOCK_4X8);
                make_block(rng, r, c + 1, AV1R_BLOCK_4X8);
            }
            return;
        }
        int k = rng.uni(0, 9);
        int half = size4 / 2, quarter = size4 / 4;
        if (k < 6 || size4 == 2) {
            make_block(rng, r, c, bsize_of(sizePx, sizePx));
        } else if (k < 8) {  // PARTITION_HORZ / VERT
            if (k == 6) {
                make_block(rng, r, c, bsize_of(sizePx, sizePx / 2));
                make_block(rng, r + half, c, bsize_of(sizePx, sizePx / 2));
            } else {
                make_block(rng, r, c, bsize_of(sizePx / 2, sizePx));
                make_block(rng, r, c + half, bsize_of(sizePx / 2, sizePx));
            }
        } else if (sizePx <= 64 && sizePx >= 16) {  // PARTITION_HORZ_4 / VERT_4
            for (int i = 0; i < 4; i++) {
                if (k == 8) make_block(rng, r + i * quarter, c, bsize_of(sizePx, sizePx / 4));
                else make_block(rng, r, c + i * quarter, bsize_of(sizePx / 4, sizePx));
            }
        } else {
            make_block(rng, r, c, bsize_of(sizePx, sizePx));
        }
    }

    void finish_filters(Rng& rng)
    {
        cdef.assign((size_t)hdr.cdef_rows * hdr.cdef_cols, -1);
        for (int r = 0; r < hdr.cdef_rows; r++)
            for (int c = 0; c < hdr.cdef_cols; c++) {
                bool allSkip = true;
                for (int y = r * 16; y < std::min(miRows, r * 16 + 16) && allSkip; y++)
                    for (int x = c * 16; x < std::min(miCols, c * 16 + 16); x++)
                        if (!(M(y, x).flags & AV1R_MI_SKIP)) {
                            allSkip = false;
                            break;
                        }
                cdef[(size_t)r * hdr.cdef_cols + c] = allSkip ? -1 : (int8_t)rng.uni(0, 7);
            }
        hdr.uses_lr = 1;
        hdr.lr_type[0] = AV1R_RESTORE_WIENER;
        hdr.lr_type[1] = hdr.lr_type[2] = AV1R_RESTORE_SGRPROJ;
        lr.clear();
        for (int p = 0; p < 3; p++) {
            int sub = p ? 1 : 0;
            int us = p ? 64 : 128;
            hdr.lr_unit_size[p] = us;
            int pw = (W + sub) >> sub, ph = (H + sub) >> sub;
            hdr.lr_unit_rows[p] = std::max((ph + (us >> 1)) / us, 1);
            hdr.lr_unit_cols[p] = std::max((pw + (us >> 1)) / us, 1);
            hdr.lr_unit_off[p] = (int32_t)lr.size();
            for (int u = 0; u < hdr.lr_unit_rows[p] * hdr.lr_unit_cols[p]; u++) {
                av1r_lr_unit x;
                memset(&x, 0, sizeof(x));
                if (rng.p(50)) {
                    x.type = p ? AV1R_RESTORE_SGRPROJ : AV1R_RESTORE_WIENER;
                    const int lo[3] = {-5, -23, -17}, hi[3] = {10, 8, 46};
                    for (int pass = 0; pass < 2; pass++)
                        for (int i = 0; i < 3; i++) x.wiener[pass][i] = (int8_t)rng.uni(lo[i], hi[i]);
                    x.sgr_set = (uint8_t)rng.uni(0, 15);
                    x.sgr_xqd[0] = (int8_t)rng.uni(-96, 31);
                    x.sgr_xqd[1] = (int8_t)rng.uni(-32, 95);
                    if (av1r_sgr_params[x.sgr_set][0] == 0) x.sgr_xqd[0] = 0;
                    if (av1r_sgr_params[x.sgr_set][2] == 0) x.sgr_xqd[1] = 0;
                }
                lr.push_back(x);
            }
        }
    }

    template <class T>
    void put(const T* d, size_t n)
    {
        uint32_t len = (uint32_t)(n * sizeof(T));
        const uint8_t* b = (const uint8_t*)&len;
        rec.insert(rec.end(), b, b + 4);
        rec.insert(rec.end(), (const uint8_t*)d, (const uint8_t*)d + len);
        while (rec.size() & 3) rec.push_back(0);
    }

    void next_frame()
    {
        Rng rng(seed * 1000003ull + (uint64_t)frameNo);
        setup_frame(rng);
        int sb4 = sb128 ? 32 : 16;
        for (int tr = 0; tr < tiles_r; tr++)
            for (int tc = 0; tc < tiles_c; tc++) {
                tileR0 = tileRowStart[tr];
                tileR1 = tileRowStart[tr + 1];
                tileC0 = tileColStart[tc];
                tileC1 = tileColStart[tc + 1];
                for (int r = tileR0; r < tileR1; r += sb4)
                    for (int c = tileC0; c < tileC1; c += sb4) {
                        clear_flags(r, c);
                        partition(rng, r, c, sb4);
                    }
            }
        finish_filters(rng);
        rec.clear();
        uint32_t magic = 0x454d5246, len = 0;
        rec.insert(rec.end(), (uint8_t*)&magic, (uint8_t*)&magic + 4);
        rec.insert(rec.end(), (uint8_t*)&len, (uint8_t*)&len + 4);
        put(&hdr, 1);
        put(mi.data(), mi.size());
        put(blocks.data(), blocks.size());
        put(tbs.data(), tbs.size());
        put(coefs.data(), coefs.size());
        uint8_t nopal = 0;
        put(&nopal, 0);
        put(cdef.data(), cdef.size());
        put(lr.data(), lr.size());
        len = (uint32_t)rec.size() - 8;
        memcpy(rec.data() + 4, &len, 4);
        frameNo++;
    }
};

}  // namespace

extern "C" {

// Open a synthetic stream: width x height 4:2:0, `tiles_c` x `tiles_r` uniform tile grid
// (SB-aligned), 128x128 superblocks if sb128.  Frame 0 is a key frame; frame k > 0 is an
// inter frame.  Returns an opaque handle.
void* av1r_synth_open(int width, int height, int sb128, int tiles_c, int tiles_r, uint32_t seed)
{
    if (width <= 0 || height <= 0 || (width & 7) || (height & 7) || tiles_c < 1 || tiles_r < 1) return nullptr;
    Gen* g = new Gen;
    g->W = width;
    g->H = height;
    g->sb128 = sb128;
    g->tiles_c = tiles_c;
    g->tiles_r = tiles_r;
    g->seed = seed;
    g->miCols = 2 * ((width + 7) >> 3);
    g->miRows = 2 * ((height + 7) >> 3);
    int sb4 = sb128 ? 32 : 16;
    g->miStride = (g->miCols + sb4 - 1) / sb4 * sb4;
    g->miRowsAlloc = (g->miRows + sb4 - 1) / sb4 * sb4;
    int sbCols = g->miStride / sb4, sbRows = g->miRowsAlloc / sb4;
    for (int i = 0; i <= tiles_c; i++) g->tileColStart.push_back(std::min(g->miCols, (i * sbCols / tiles_c) * sb4));
    for (int i = 0; i <= tiles_r; i++) g->tileRowStart.push_back(std::min(g->miRows, (i * sbRows / tiles_r) * sb4));
    g->tileColStart[tiles_c] = g->miCols;
    g->tileRowStart[tiles_r] = g->miRows;
    return g;
}

// Generate the next frame; *data / *len point at its FRME record (the .av1b frame
// record of av1dec_amd/batchfile.py), valid until the next call.
int av1r_synth_next(void* h, const uint8_t** data, size_t* len)
{
    Gen* g = (Gen*)h;
    if (!g) return -1;
    g->next_frame();
    *data = g->rec.data();
    *len = g->rec.size();
    return 0;
}

void av1r_synth_close(void* h) { delete (Gen*)h; }

}  // extern "C"
