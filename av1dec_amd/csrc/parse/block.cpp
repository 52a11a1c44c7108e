// block.cpp -- tile / superblock / partition / block / transform-block syntax of the host
// parser, emitting the av1r batch records (include/av1r.h) as it goes.
//
// One pass per tile: the reference parses a whole tile into its object tree
// (Tile::parse, decoder/Tile.cpp:122-160) and reconstructs afterwards; what the batch needs
// from reconstruction time (BlockDecoded flags, LoopfilterTxSizes, MaxLumaW/H, the local warp
// fit) only depends on blocks earlier in decode order, so it is computed right after each
// block's syntax here.  Reference behaviour restated (oddstone/av1dec, decoder/):
//   Partition::parse                     Partition.cpp:127-205, 230-259
//   Block::Block / parse / residual      Block.cpp:46-88, 176-363
//   mode info (intra / inter)            Block.cpp:365-1465
//   tx size / var tx                     Block.cpp:1468-1598
//   ref frames                           Block.cpp:1618-1936
//   palette                              Block.cpp:1938-2271
//   local warp                           Block.cpp:946-1200
//   FindMvStack                          InterPredict.cpp:1051-1669
//   TransformBlock parse / coeffs        TransformBlock.cpp:1165-1704, 2278-2374
//   decode-time flags                    TransformBlock.cpp:2376-2456, Tile.cpp:41-90
//   CDEF / LR syntax                     Parser.cpp:2007-2023, 2112-2225
//   batch assembly                       oracle/harness/refdump.cpp dumpBlock
// Where the reference reads outside the arrays it allocated (K5 in SURVEY.md) this file
// keeps to the specification's bounds.
#include <stdlib.h>

#include <algorithm>

#include "parser.h"
#include "scan_tables.h"

namespace av1p {
namespace {

enum { BLOCK_4X4 = 0, BLOCK_8X8 = 3, BLOCK_32X32 = 9, BLOCK_64X64 = 12, BLOCK_128X128 = 15 };
enum { TX_4X4 = 0, TX_32X32 = 3, TX_64X64 = 4, TX_16X32 = 9, TX_32X16 = 10, TX_16X64 = 17, TX_64X16 = 18 };
enum { DC_PRED = 0, V_PRED = 1, D67_PRED = 8, SMOOTH_PRED = 9, SMOOTH_V_PRED = 10, SMOOTH_H_PRED = 11,
       NEARESTMV = 13, NEARMV, GLOBALMV, NEWMV, NEAREST_NEARESTMV, NEAR_NEARMV, NEAREST_NEWMV, NEW_NEARESTMV,
       NEAR_NEWMV, NEW_NEARMV, GLOBAL_GLOBALMV, NEW_NEWMV };
enum { UV_CFL_PRED = 13 };
enum { SIMPLE_TRANSLATION = 0, OBMC_CAUSAL = 1, LOCALWARP = 2 };
enum { COMPOUND_WEDGE = 0, COMPOUND_DIFFWTD = 1, COMPOUND_AVERAGE = 2, COMPOUND_INTRA = 3, COMPOUND_DISTANCE = 4 };
enum { EIGHTTAP = 0, BILINEAR = 3 };
enum { GM_IDENTITY = 0, GM_TRANSLATION = 1 };
enum { DCT_DCT = 0, ADST_DCT, DCT_ADST, ADST_ADST, FLIPADST_DCT, DCT_FLIPADST, FLIPADST_FLIPADST, ADST_FLIPADST,
       FLIPADST_ADST, IDTX, V_DCT, H_DCT, V_ADST, H_ADST, V_FLIPADST, H_FLIPADST };

// ---- specification tables (AV1 spec, Additional tables) ----
const uint8_t kMaxTxSizeRect[22] = {0, 5, 6, 1, 7, 8, 2, 9, 10, 3, 11, 12, 4, 4, 4, 4, 13, 14, 15, 16, 17, 18};
const uint8_t kMaxTxDepth[22] = {0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 4, 4, 4, 4, 4, 4, 2, 2, 3, 3, 4, 4};
const uint8_t kSplitTxSize[19] = {0, 0, 1, 2, 3, 0, 0, 1, 1, 2, 2, 3, 3, 5, 6, 7, 8, 9, 10};
const uint8_t kTxSizeSqr[19] = {0, 1, 2, 3, 4, 0, 0, 1, 1, 2, 2, 3, 3, 0, 0, 1, 1, 2, 2};
const uint8_t kTxSizeSqrUp[19] = {0, 1, 2, 3, 4, 1, 1, 2, 2, 3, 3, 4, 4, 2, 2, 3, 3, 4, 4};
const uint8_t kAdjustedTxSize[19] = {0, 1, 2, 3, 3, 5, 6, 7, 8, 9, 10, 3, 3, 13, 14, 15, 16, 9, 10};
const uint8_t kSizeGroup[22] = {0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 0, 0, 1, 1, 2, 2};
const uint8_t kIntraModeContext[13] = {0, 1, 2, 3, 4, 4, 4, 4, 3, 0, 1, 2, 0};
// Partition_Subsize for the square sizes 8x8 .. 128x128 (index = log2(size) - 3)
const int8_t kSubsize[10][5] = {
    {3, 6, 9, 12, 15},     {2, 5, 8, 11, 14},     {1, 4, 7, 10, 13},     {0, 3, 6, 9, 12},
    {2, 5, 8, 11, 14},     {2, 5, 8, 11, 14},     {1, 4, 7, 10, 13},     {1, 4, 7, 10, 13},
    {-1, 17, 19, 21, -1},  {-1, 16, 18, 20, -1}};
const uint8_t kTxInSetIntra[3][16] = {{1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
                                      {1, 1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 1, 0, 0, 0, 0},
                                      {1, 1, 1, 1, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0}};
const uint8_t kTxInSetInter[4][16] = {{1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
                                      {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1},
                                      {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0},
                                      {1, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0}};
const uint8_t kModeToTxfm[14] = {DCT_DCT,  ADST_DCT,  DCT_ADST,  DCT_DCT,  ADST_ADST, ADST_DCT,  DCT_ADST,
                                 DCT_ADST, ADST_DCT,  ADST_ADST, ADST_DCT, DCT_ADST,  ADST_ADST, DCT_DCT};
const uint8_t kFilterIntraModeToIntraDir[5] = {DC_PRED, V_PRED, 2 /*H_PRED*/, 6 /*D157_PRED*/, DC_PRED};
const uint8_t kIntraInvSet1[7] = {IDTX, DCT_DCT, V_DCT, H_DCT, ADST_ADST, ADST_DCT, DCT_ADST};
const uint8_t kIntraInvSet2[5] = {IDTX, DCT_DCT, ADST_ADST, ADST_DCT, DCT_ADST};
const uint8_t kInterInvSet1[16] = {IDTX,      V_DCT,        H_DCT,     V_ADST,    H_ADST,   V_FLIPADST,
                                   H_FLIPADST, DCT_DCT,     ADST_DCT,  DCT_ADST,  FLIPADST_DCT, DCT_FLIPADST,
                                   ADST_ADST, FLIPADST_FLIPADST, ADST_FLIPADST, FLIPADST_ADST};
const uint8_t kInterInvSet2[12] = {IDTX,     V_DCT,        H_DCT,        DCT_DCT,   ADST_DCT,          DCT_ADST,
                                   FLIPADST_DCT, DCT_FLIPADST, ADST_ADST, FLIPADST_FLIPADST, ADST_FLIPADST, FLIPADST_ADST};
const int8_t kSigRefDiffOffset[3][5][2] = {{{0, 1}, {1, 0}, {1, 1}, {0, 2}, {2, 0}},
                                           {{0, 1}, {1, 0}, {0, 2}, {0, 3}, {0, 4}},
                                           {{0, 1}, {1, 0}, {2, 0}, {3, 0}, {4, 0}}};
const int8_t kMagRefOffset[3][3][2] = {{{0, 1}, {1, 0}, {1, 1}}, {{0, 1}, {1, 0}, {0, 2}}, {{0, 1}, {1, 0}, {2, 0}}};
const uint8_t kCoeffBasePosCtxOffset[3] = {26, 31, 36};
const int8_t kPaletteColorContext[9] = {-1, -1, 0, -1, -1, 4, 3, 2, 1};
const uint8_t kCompoundModeCtxMap[3][5] = {{0, 1, 1, 1, 1}, {1, 2, 3, 4, 4}, {4, 4, 5, 6, 7}};
const int kWienerTapsMin[3] = {-5, -23, -17};
const int kWienerTapsMax[3] = {10, 8, 46};
const int kWienerTapsK[3] = {1, 2, 3};
const int kWienerTapsMid[3] = {3, -7, 15};
const int kSgrprojXqdMin[2] = {-96, -32};
const int kSgrprojXqdMax[2] = {31, 95};
const int kSgrprojXqdMid[2] = {-32, 31};

constexpr int kRefCatLevel640 = 640;
constexpr int kSigCoefContexts = 42, kSigCoefContextsEob = 4;
constexpr int kNumBaseLevels = 2, kCoeffBaseRange = 12, kBrCdfSize = 4;

inline int bw4_of(int bs) { return av1r_num4x4w[bs]; }
inline int bh4_of(int bs) { return av1r_num4x4h[bs]; }
inline int clip3(int lo, int hi, int v) { return v < lo ? lo : v > hi ? hi : v; }
inline int round2(int64_t x, int n) { return n == 0 ? (int)x : (int)((x + ((int64_t)1 << (n - 1))) >> n); }
inline int64_t round2_64(int64_t x, int n) { return n == 0 ? x : (x + ((int64_t)1 << (n - 1))) >> n; }
inline int64_t round2signed_64(int64_t x, int n) { return x >= 0 ? round2_64(x, n) : -round2_64(-x, n); }
inline bool directional(int mode) { return mode >= V_PRED && mode <= D67_PRED; }
inline int floor_log2(uint64_t x)
{
    int s = 0;
    while (x > 1) {
        x >>= 1;
        s++;
    }
    return s;
}
inline int ceil_log2(uint32_t x)
{
    if (x < 2) return 0;
    int i = 1;
    uint32_t p = 2;
    while (p < x) {
        i++;
        p <<= 1;
    }
    return i;
}
inline int find_tx_size(int w, int h)
{
    for (int t = 0; t < AV1R_TX_SIZES; t++)
        if (av1r_tx_w[t] == w && av1r_tx_h[t] == h) return t;
    return AV1R_TX_SIZES;
}

const int16_t* default_scan(int tx)
{
    switch (tx) {
    case 0: return kDefaultScan4x4;
    case 5: return kDefaultScan4x8;
    case 6: return kDefaultScan8x4;
    case 1: return kDefaultScan8x8;
    case 7: return kDefaultScan8x16;
    case 8: return kDefaultScan16x8;
    case 2: return kDefaultScan16x16;
    case 9: return kDefaultScan16x32;
    case 10: return kDefaultScan32x16;
    case 13: return kDefaultScan4x16;
    case 14: return kDefaultScan16x4;
    case 15: return kDefaultScan8x32;
    case 16: return kDefaultScan32x8;
    default: return kDefaultScan32x32;
    }
}
const int16_t* mrow_scan(int tx)
{
    switch (tx) {
    case 0: return kMrowScan4x4;
    case 5: return kMrowScan4x8;
    case 6: return kMrowScan8x4;
    case 1: return kMrowScan8x8;
    case 7: return kMrowScan8x16;
    case 8: return kMrowScan16x8;
    case 2: return kMrowScan16x16;
    case 13: return kMrowScan4x16;
    default: return kMrowScan16x4;
    }
}
const int16_t* mcol_scan(int tx)
{
    switch (tx) {
    case 0: return kMcolScan4x4;
    case 5: return kMcolScan4x8;
    case 6: return kMcolScan8x4;
    case 1: return kMcolScan8x8;
    case 7: return kMcolScan8x16;
    case 8: return kMcolScan16x8;
    case 2: return kMcolScan16x16;
    case 13: return kMcolScan4x16;
    default: return kMcolScan16x4;
    }
}
// TransformBlock::get_scan (TransformBlock.cpp:1402-1424)
const int16_t* get_scan(int tx, int type)
{
    if (tx == TX_16X64) return kDefaultScan16x32;
    if (tx == TX_64X16) return kDefaultScan32x16;
    if (kTxSizeSqrUp[tx] == TX_64X64) return kDefaultScan32x32;
    if (type == IDTX) return default_scan(tx);
    if (type == V_DCT || type == V_ADST || type == V_FLIPADST) return mrow_scan(tx);
    if (type == H_DCT || type == H_ADST || type == H_FLIPADST) return mcol_scan(tx);
    return default_scan(tx);
}
int tx_class(int type)
{
    if (type == V_DCT || type == V_ADST || type == V_FLIPADST) return TX_CLASS_VERT;
    if (type == H_DCT || type == H_ADST || type == H_FLIPADST) return TX_CLASS_HORIZ;
    return TX_CLASS_2D;
}

// Per scan position of a transform size and class, everything the level loop of coeffs()
// derives from the position (built once): its offset in the padded level map, its raster
// position, the base-level context offset (kCoeffBaseCtxOffset / kCoeffBasePosCtxOffset;
// bit 7: the DC of a 2D class, whose context is 0) and the range context offset (0 / 7 / 14,
// TransformBlock::get_br_ctx).  The scan orders and offsets are the spec's
// (TransformBlock.cpp:1402-1424, 1462-1580).
struct ScanEntry {
    uint16_t pad, pos;
    uint8_t base, br;
};
struct ScanTables {
    std::vector<ScanEntry> t[19][3];  // [tx size][class]
    ScanTables()
    {
        static const int kTypeOfClass[3] = {DCT_DCT, H_DCT, V_DCT};  // TX_CLASS_2D / HORIZ / VERT
        for (int tx = 0; tx < 19; tx++)
            for (int cls = 0; cls < 3; cls++) {
                // (the 1D classes -- V_* / H_* types -- only in transform sets of sizes up to 16x16)
                if (cls != TX_CLASS_2D && kTxSizeSqrUp[tx] > 2) continue;
                const int16_t* scan = get_scan(tx, kTypeOfClass[cls]);
                const int adj = kAdjustedTxSize[tx];
                const int bwl = av1r_tx_w_log2[adj], width = 1 << bwl, height = av1r_tx_h[adj], ps = width + 4;
                std::vector<ScanEntry>& v = t[tx][cls];
                v.resize((size_t)height << bwl);
                for (size_t c = 0; c < v.size(); c++) {
                    const int pos = scan[c], row = pos >> bwl, col = pos - (row << bwl);
                    ScanEntry& e = v[c];
                    e.pad = (uint16_t)(row * ps + col);
                    e.pos = (uint16_t)pos;
                    if (cls == TX_CLASS_2D) e.base = pos == 0 ? 0x80 : kCoeffBaseCtxOffset[tx][std::min(row, 4)][std::min(col, 4)];
                    else e.base = kCoeffBasePosCtxOffset[std::min(cls == TX_CLASS_VERT ? row : col, 2)];
                    if (pos == 0) e.br = 0;
                    else if (cls == TX_CLASS_2D) e.br = (row < 2 && col < 2) ? 7 : 14;
                    else if (cls == TX_CLASS_HORIZ) e.br = col == 0 ? 7 : 14;
                    else e.br = row == 0 ? 7 : 14;
                }
            }
    }
};
const ScanTables kScanTables;

// ---- per-block parse state (the members of the reference's Block, Block.h:198-275) ----
struct Blk {
    int r, c, bsize, bw4, bh4;
    bool has_chroma, avail_u, avail_l, avail_u_uv, avail_l_uv;
    bool is_inter = false, use_intrabc = false, skip = false, skip_mode = false, lossless = false;
    int y_mode = 0, uv_mode = 0, angle_y = 0, angle_uv = 0, cfl_u = 0, cfl_v = 0;
    int pal_y = 0, pal_uv = 0;
    uint8_t colors[3][8] = {};
    bool use_filter_intra = false;
    int filter_intra_mode = 0;
    int tx_size = 0;
    int ref[2] = {0, -1};
    int qindex = 0;
    // inter
    int left_ref[2] = {0, -1}, above_ref[2] = {0, -1};
    bool left_intra = false, above_intra = false, left_single = false, above_single = false;
    int ref_mv_idx = 0;
    Mv mv[2];
    bool interintra = false, wedge_interintra = false;
    int interintra_mode = 0, wedge_index = 0, wedge_sign = 0;
    int motion_mode = 0, compound_type = COMPOUND_AVERAGE;
    bool comp_group_idx = false, compound_idx = true, mask_type = false;
    int interp[2] = {0, 0};
    // local warp (Block::LocalWarp)
    int num_samples = 0, num_scanned = 0;
    int cand[9][4] = {};
    bool local_valid = false;
    int32_t local_warp[6] = {};
    // palette maps (Block::Palette)
    int map_wy = 0, map_hy = 0, map_wuv = 0, map_huv = 0;
    std::vector<uint8_t> map_y, map_uv;
};

// one parsed transform block, kept until the block's records are emitted
struct Tb {
    int plane, x, y, base_x, base_y, tx;
    int eob;
    int type;
    uint32_t coef_off, coef_cnt;
};

// ---- FindMvStack state (InterPredict.cpp:1051-1669) ----
struct MvStack {
    int num = 0, new_count = 0;
    bool found = false;
    Mv stack[kMaxRefMvStack + 1][2];
    uint32_t weight[kMaxRefMvStack + 1] = {};
    Mv global[2];
    int new_ctx = 0, ref_ctx = 0, zero_ctx = 0;
    uint8_t drl_ctx[kMaxRefMvStack + 1] = {};
};

// extraSearch's candidate lists: never more than 2 entries, kept on the stack
struct MvList2 {
    Mv v[2];
    size_t n = 0;
    size_t size() const { return n; }
    void push_back(const Mv& m) { v[n++] = m; }
    const Mv& operator[](size_t i) const { return v[i]; }
    const Mv* begin() const { return v; }
    const Mv* end() const { return v + n; }
};

class BlockParser {
public:
    BlockParser(Parser& p, TileCtx& t) : P(p), T(t), fh(p.fh), seq(p.seq), sd(t.sd), cdf(t.tcdf) {}
    void decode_partition(int r, int c, int bsize);
    void read_lr(int r, int c, int bsize);

private:
    Parser& P;
    TileCtx& T;
    const FrameHdr& fh;
    const SeqHdr& seq;
    SymbolDecoder& sd;
    Cdfs& cdf;
    std::vector<Tb> tbs;
    std::vector<int> quant;  // Quant[] of the transform block being parsed
    // coefficient levels while parsing them, padded (coeffs()): level << 8 | min(level, 3)
    uint16_t lvl[36 * 36] = {};
    uint16_t nzc[1024];  // the scan indices of a transform block's non-zero levels, last first

    int S(uint16_t* c, int n) { return sd.read(c, n); }  // (SymbolDecoder::read dispatches every alphabet size 2..16 to readN<N>: measured faster, 3a5ab10)
    template <int N>
    int SN(uint16_t* c) { return sd.readN<N>(c); }
    uint32_t L(int n) { return sd.literal(n); }
    MiInfo& mi(int r, int c) { return P.mi_at(r, c); }
    bool inside(int r, int c) const { return T.is_inside(r, c); }

    void decode_block(int r, int c, int bsize);
    // mode info
    void intra_frame_mode_info(Blk& b);
    void inter_frame_mode_info(Blk& b);
    void intra_block_mode_info(Blk& b);
    void inter_block_mode_info(Blk& b);
    bool read_skip(Blk& b);
    void read_cdef(Blk& b);
    void read_delta_qindex(Blk& b);
    void read_delta_lf(Blk& b);
    void intra_angle_info_y(Blk& b);
    void read_uv_mode(Blk& b);
    void read_cfl_alphas(Blk& b);
    void filter_intra_mode_info(Blk& b);
    void read_ref_frames(Blk& b);
    void read_comp_reference(Blk& b);
    void read_single_reference(Blk& b);
    int count_refs(const Blk& b, int type) const;
    void assign_mv(Blk& b, const MvStack& s, bool isCompound);
    void read_mv(Blk& b, const Mv* pred, int ref);
    int read_mv_component(int ctx, int comp);
    void read_interintra_mode(Blk& b, bool isCompound);
    void read_motion_mode(Blk& b, bool isCompound);
    void read_compound_type(Blk& b, bool isCompound);
    bool has_overlappable_candidates(const Blk& b);
    bool needs_interp_filter(const Blk& b) const;
    int interp_filter_ctx(const Blk& b, int dir);
    bool is_scaled(int refFrame) const;
    // mv stack
    void find_mv_stack(Blk& b, MvStack& s);
    void setup_global_mv(const Blk& b, MvStack& s, int refList);
    void lower_mv_precision(Mv& mv) const;
    void scan_row(const Blk& b, MvStack& s, int deltaRow);
    void scan_col(const Blk& b, MvStack& s, int deltaCol);
    void scan_point(const Blk& b, MvStack& s, int deltaRow, int deltaCol);
    void add_ref_mv_candidate(const Blk& b, MvStack& s, int mvRow, int mvCol, uint32_t weight);
    void search_stack(const Blk& b, MvStack& s, int mvRow, int mvCol, int candList, uint32_t weight);
    void search_compound_stack(const Blk& b, MvStack& s, int mvRow, int mvCol, uint32_t weight);
    void temporal_scan(const Blk& b, MvStack& s);
    void extra_search(const Blk& b, MvStack& s);
    void add_extra_mv_candidate(const Blk& b, MvStack& s, int mvRow, int mvCol, MvList2* idMvs, MvList2* diffMvs);
    // local warp
    void find_warp_samples(Blk& b);
    void add_sample(Blk& b, int deltaRow, int deltaCol);
    void warp_estimation(Blk& b);
    // palette
    void palette_mode_info(Blk& b);
    int palette_cache(const Blk& b, int plane, uint8_t* cache);
    void palette_tokens(Blk& b);
    // transform sizes and residual
    void read_block_tx_size(Blk& b);
    void read_tx_size(Blk& b, bool allowSelect);
    void read_var_tx_size(Blk& b, int row, int col, int txSz, int depth);
    int above_tx_width(const Blk& b, int row, int col);
    int left_tx_height(const Blk& b, int row, int col);
    void reset_block_context(const Blk& b);
    void residual(Blk& b);
    void transform_tree(Blk& b, int startX, int startY, int w, int h);
    void transform_block(Blk& b, int plane, int baseX, int baseY, int txSz, int x, int y);
    int uv_tx_size(const Blk& b) const;
    int tx_set(const Blk& b, int txSz) const;
    int compute_tx_type(const Blk& b, int plane, int txSz, int x4, int y4) const;
    int coeffs(Blk& b, Tb& t);
    int all_zero_ctx(const Blk& b, int plane, int txSz, int x4, int y4, int w, int h) const;
    // batch emission
    void emit(Blk& b);
    bool flag(int plane, int r, int c) const { return T.decoded[plane][r + 1][c + 1] != 0; }
};

// ------------------------------------------------------------------------------------
// partition (Partition.cpp:127-259)
// ------------------------------------------------------------------------------------
void BlockParser::decode_partition(int r, int c, int bsize)
{
    if (r >= fh.mi_rows || c >= fh.mi_cols || !T.err.empty()) return;
    const int num4x4 = bw4_of(bsize);
    const int half = num4x4 >> 1, quarter = half >> 1;
    const bool hasRows = (r + half) < fh.mi_rows;
    const bool hasCols = (c + half) < fh.mi_cols;
    int partition;
    if (bsize < BLOCK_8X8) {
        partition = PARTITION_NONE;
    } else {
        const bool availU = inside(r - 1, c), availL = inside(r, c - 1);
        const int bsl = av1r_miw_log2[bsize];
        const int above = availU && av1r_miw_log2[mi(r - 1, c).mi_size] < bsl;
        const int left = availL && av1r_mih_log2[mi(r, c - 1).mi_size] < bsl;
        const int ctx = left * 2 + above;
        uint16_t* pc = cdf.mode.partition[(bsl - 1) * 4 + ctx];
        const int nsym = bsl == 1 ? 4 : bsl == 5 ? 8 : 10;
        if (hasRows && hasCols) {
            partition = S(pc, nsym);
        } else if (hasCols || hasRows) {
            // split_or_horz / split_or_vert (EntropyDecoder.cpp:75-97): a boolean whose
            // probability sums the partition CDF's split-like symbols; never adapted
            auto p = [&](int s) { return (int)pc[s] - (int)pc[s - 1]; };  // = -P(s), inverted CDF
            int psum;
            if (hasCols) {
                psum = p(PARTITION_VERT) + p(PARTITION_SPLIT) + p(PARTITION_HORZ_A) + p(PARTITION_VERT_A) + p(PARTITION_VERT_B);
                if (bsize != BLOCK_128X128) psum += p(PARTITION_VERT_4);
            } else {
                psum = p(PARTITION_HORZ) + p(PARTITION_SPLIT) + p(PARTITION_HORZ_A) + p(PARTITION_HORZ_B) + p(PARTITION_VERT_A);
                if (bsize != BLOCK_128X128) psum += p(PARTITION_HORZ_4);
            }
            uint16_t icdf[3] = {(uint16_t)(-psum), 0, 0};
            const bool nu = sd.noUpdate;
            sd.noUpdate = true;
            const bool split = sd.read(icdf, 2) != 0;
            sd.noUpdate = nu;
            partition = split ? PARTITION_SPLIT : hasCols ? PARTITION_HORZ : PARTITION_VERT;
        } else {
            partition = PARTITION_SPLIT;
        }
    }
    const int lvl = av1r_miw_log2[bsize] - 1;  // 8x8 -> 0 .. 128x128 -> 4
    const int subSize = bsize < BLOCK_8X8 ? bsize : kSubsize[partition][lvl];
    const int splitSize = bsize < BLOCK_8X8 ? bsize : kSubsize[PARTITION_SPLIT][lvl];
    if (subSize < 0) {
        T.fail(AV1R_E_INVALID, "invalid partition %d for block size %d", partition, bsize);
        return;
    }
    switch (partition) {
    case PARTITION_NONE: decode_block(r, c, subSize); break;
    case PARTITION_HORZ:
        decode_block(r, c, subSize);
        if (hasRows) decode_block(r + half, c, subSize);
        break;
    case PARTITION_VERT:
        decode_block(r, c, subSize);
        if (hasCols) decode_block(r, c + half, subSize);
        break;
    case PARTITION_SPLIT:
        decode_partition(r, c, subSize);
        decode_partition(r, c + half, subSize);
        decode_partition(r + half, c, subSize);
        decode_partition(r + half, c + half, subSize);
        break;
    case PARTITION_HORZ_A:
        decode_block(r, c, splitSize);
        decode_block(r, c + half, splitSize);
        decode_block(r + half, c, subSize);
        break;
    case PARTITION_HORZ_B:
        decode_block(r, c, subSize);
        decode_block(r + half, c, splitSize);
        decode_block(r + half, c + half, splitSize);
        break;
    case PARTITION_VERT_A:
        decode_block(r, c, splitSize);
        decode_block(r + half, c, splitSize);
        decode_block(r, c + half, subSize);
        break;
    case PARTITION_VERT_B:
        decode_block(r, c, subSize);
        decode_block(r, c + half, splitSize);
        decode_block(r + half, c + half, splitSize);
        break;
    case PARTITION_HORZ_4:
        for (int i = 0; i < 4; i++)
            if (i < 3 || r + quarter * 3 < fh.mi_rows) decode_block(r + quarter * i, c, subSize);
        break;
    default:
        for (int i = 0; i < 4; i++)
            if (i < 3 || c + quarter * 3 < fh.mi_cols) decode_block(r, c + quarter * i, subSize);
        break;
    }
}

// ------------------------------------------------------------------------------------
// block (Block::Block + Block::parse, Block.cpp:46-88, 313-363)
// ------------------------------------------------------------------------------------
#ifdef AV1P_PROF  // debug aid: cycles per phase of the block walk, printed at exit
#include <x86intrin.h>
struct ProfAcc {
    uint64_t t[10] = {};
    ~ProfAcc()
    {
        fprintf(stderr, "av1p prof (Mcycles): mode %.1f residual %.1f mi %.1f emit %.1f | coef %.1f: head %.1f eob %.1f levels %.1f signs %.1f pack %.1f\n",
                t[0] / 1e6, t[1] / 1e6, t[2] / 1e6, t[3] / 1e6, t[9] / 1e6, t[4] / 1e6, t[5] / 1e6, t[6] / 1e6, t[7] / 1e6, t[8] / 1e6);
    }
};
static ProfAcc g_prof;
#define PROF_T(v) const uint64_t v = __rdtsc()
#define PROF_ADD(i, a, b) g_prof.t[i] += (b) - (a)
#else
#define PROF_T(v)
#define PROF_ADD(i, a, b)
#endif

void BlockParser::decode_block(int r, int c, int bsize)
{
    if (!T.err.empty()) return;
    Blk b;
    b.r = r;
    b.c = c;
    b.bsize = bsize;
    b.bw4 = bw4_of(bsize);
    b.bh4 = bh4_of(bsize);
    if (b.bh4 == 1 && (r & 1) == 0) b.has_chroma = false;
    else if (b.bw4 == 1 && (c & 1) == 0) b.has_chroma = false;
    else b.has_chroma = true;
    b.avail_u = inside(r - 1, c);
    b.avail_l = inside(r, c - 1);
    b.avail_u_uv = b.avail_u;
    b.avail_l_uv = b.avail_l;
    if (b.has_chroma) {
        if (b.bh4 == 1) b.avail_u_uv = inside(r - 2, c);
        if (b.bw4 == 1) b.avail_l_uv = inside(r, c - 2);
    } else {
        b.avail_u_uv = b.avail_l_uv = false;
    }
    b.qindex = T.current_q;
    tbs.clear();

    PROF_T(t0);
    if (fh.frame_is_intra) intra_frame_mode_info(b);
    else inter_frame_mode_info(b);
    palette_tokens(b);
    read_block_tx_size(b);
    if (b.skip) reset_block_context(b);
    const bool isCompound = b.ref[1] > INTRA_FRAME;
    PROF_T(t1);
    PROF_ADD(0, t0, t1);
    uint32_t palIdx = ~0u;
    if (b.pal_y || b.pal_uv) {
        palIdx = (uint32_t)T.pal_colors.size();
        std::vector<uint8_t> cols(16, 0);
        for (int i = 0; i < b.pal_y; i++) cols[i] = b.colors[0][i];
        for (int i = 0; i < b.pal_uv; i++) cols[8 + i] = b.colors[1][i];
        T.pal_colors.push_back(cols);
    }
    // the block's mode info into every 4x4 unit it covers, in one pass (the residual below
    // reads only the units' transform sizes and types)
    for (int y = 0; y < b.bh4; y++) {
        MiInfo* row = &mi(r + y, c);
        for (int x = 0; x < b.bw4; x++) {
            MiInfo& m = row[x];
            m.y_mode = (uint8_t)b.y_mode;
            if (b.ref[0] == INTRA_FRAME && b.has_chroma) m.uv_mode = (uint8_t)b.uv_mode;
            m.ref[0] = (int8_t)b.ref[0];
            m.ref[1] = (int8_t)b.ref[1];
            if (b.is_inter) {
                if (!b.use_intrabc) {
                    m.comp_group_idx = b.comp_group_idx;
                    m.compound_idx = b.compound_idx;
                }
                m.interp[0] = (uint8_t)b.interp[0];
                m.interp[1] = (uint8_t)b.interp[1];
                for (int l = 0; l < 1 + isCompound; l++) m.mv[l] = b.mv[l];
            }
            m.is_inter = b.is_inter;
            m.skip_mode = b.skip_mode;
            m.skip = b.skip;
            m.mi_size = (uint8_t)bsize;
            m.pal_size[0] = (uint8_t)b.pal_y;
            m.pal_size[1] = (uint8_t)b.pal_uv;
            m.pal_idx = palIdx;
        }
        if (P.emit_mi)
            for (int x = 0; x < b.bw4; x++)
                for (int i = 0; i < 4; i++) P.mi_dlf[((size_t)(r + y) * P.mi_stride + c + x) * 4 + i] = (int8_t)T.delta_lf[i];
    }
    PROF_T(t2);
    residual(b);
    PROF_T(t3);
    PROF_ADD(2, t1, t2);
    PROF_ADD(1, t2, t3);
    if (!T.err.empty()) return;
    PROF_T(t4);
    emit(b);
    PROF_T(t5);
    PROF_ADD(3, t4, t5);
}

bool BlockParser::read_skip(Blk& b)
{
    int ctx = 0;
    if (b.avail_u) ctx += mi(b.r - 1, b.c).skip;
    if (b.avail_l) ctx += mi(b.r, b.c - 1).skip;
    return S(cdf.mode.skip[ctx], 2) != 0;
}

// read_cdef (Block.cpp:381-386, Parser.cpp:2007-2023); the grid is kept per 64x64
void BlockParser::read_cdef(Blk& b)
{
    if (b.skip || fh.coded_lossless || !seq.enable_cdef || fh.allow_intrabc) return;
    const int r = b.r & ~15, c = b.c & ~15;
    int8_t& cur = P.cdef_idx[(size_t)(r >> 4) * P.cdef_cols + (c >> 4)];
    if (cur != -1) return;
    const int idx = (int)L(fh.cdef_bits);
    for (int i = r; i < r + b.bh4; i += 16)
        for (int j = c; j < c + b.bw4; j += 16)
            if ((i >> 4) < P.cdef_rows && (j >> 4) < P.cdef_cols) P.cdef_idx[(size_t)(i >> 4) * P.cdef_cols + (j >> 4)] = (int8_t)idx;
}

void BlockParser::read_delta_qindex(Blk& b)
{
    const int sbSize = seq.use_128x128 ? BLOCK_128X128 : BLOCK_64X64;
    if (b.bsize == sbSize && b.skip) return;
    if (!T.read_deltas) return;
    int abs = S(cdf.mode.delta_q, 4);
    if (abs == 3) {
        const int remBits = (int)L(3) + 1;
        abs = (int)L(remBits) + (1 << remBits) + 1;
    }
    if (abs) {
        const int sign = (int)L(1);
        const int reduced = sign ? -abs : abs;
        T.current_q = clip3(1, 255, T.current_q + reduced * (1 << fh.delta_q_res));
        b.qindex = T.current_q;
    }
}

void BlockParser::read_delta_lf(Blk& b)
{
    const int sbSize = seq.use_128x128 ? BLOCK_128X128 : BLOCK_64X64;
    if (b.bsize == sbSize && b.skip) return;
    if (!(T.read_deltas && fh.delta_lf_present)) return;
    const int count = fh.delta_lf_multi ? 4 : 1;
    for (int i = 0; i < count; i++) {
        int abs = S(fh.delta_lf_multi ? cdf.mode.delta_lf_multi[i] : cdf.mode.delta_lf, 4);
        if (abs == 3) {
            const int n = (int)L(3) + 1;
            abs = (int)L(n) + (1 << n) + 1;
        }
        if (abs) {
            const int sign = (int)L(1);
            const int reduced = sign ? -abs : abs;
            T.delta_lf[i] = clip3(-63, 63, T.delta_lf[i] + reduced * (1 << fh.delta_lf_res));
        }
    }
}

void BlockParser::intra_angle_info_y(Blk& b)
{
    if (b.bsize >= BLOCK_8X8 && directional(b.y_mode)) b.angle_y = S(cdf.mode.angle_delta[b.y_mode - V_PRED], 7) - 3;
}

void BlockParser::read_uv_mode(Blk& b)
{
    bool cflAllowed;
    if (b.lossless && av1r_ss420[b.bsize] == BLOCK_4X4) cflAllowed = true;
    else if (!b.lossless && std::max(b.bw4, b.bh4) <= 8) cflAllowed = true;
    else cflAllowed = false;
    b.uv_mode = S(cdf.mode.uv_mode[cflAllowed][b.y_mode], cflAllowed ? 14 : 13);
    if (b.uv_mode == UV_CFL_PRED) read_cfl_alphas(b);
    if (b.bsize >= BLOCK_8X8 && directional(b.uv_mode)) b.angle_uv = S(cdf.mode.angle_delta[b.uv_mode - V_PRED], 7) - 3;
}

void BlockParser::read_cfl_alphas(Blk& b)
{
    static const int ctxV[8] = {0, 3, 0, 1, 4, 0, 2, 5};
    const int signs = S(cdf.mode.cfl_sign, 8);
    const int signU = (signs + 1) / 3, signV = (signs + 1) % 3;
    b.cfl_u = 0;
    b.cfl_v = 0;
    if (signU) {
        b.cfl_u = S(cdf.mode.cfl_alpha[signs - 2], 16) + 1;
        if (signU == 1) b.cfl_u = -b.cfl_u;
    }
    if (signV) {
        b.cfl_v = S(cdf.mode.cfl_alpha[ctxV[signs]], 16) + 1;
        if (signV == 1) b.cfl_v = -b.cfl_v;
    }
}

void BlockParser::filter_intra_mode_info(Blk& b)
{
    b.use_filter_intra = false;
    if (seq.enable_filter_intra && b.y_mode == DC_PRED && b.pal_y == 0 && std::max(b.bw4, b.bh4) <= 8) {
        b.use_filter_intra = S(cdf.mode.filter_intra[b.bsize], 2) != 0;
        if (b.use_filter_intra) b.filter_intra_mode = S(cdf.mode.filter_intra_mode, 5);
    }
}

// intra_frame_mode_info (Block.cpp:534-593)
void BlockParser::intra_frame_mode_info(Blk& b)
{
    b.skip_mode = false;
    b.skip = read_skip(b);
    b.lossless = fh.coded_lossless;
    read_cdef(b);
    read_delta_qindex(b);
    read_delta_lf(b);
    T.read_deltas = false;
    b.ref[0] = INTRA_FRAME;
    b.ref[1] = NONE_FRAME;
    b.use_intrabc = fh.allow_intrabc ? S(cdf.mode.intrabc, 2) != 0 : false;
    if (b.use_intrabc) {
        b.is_inter = true;
        b.y_mode = DC_PRED;
        b.uv_mode = 0;
        b.motion_mode = SIMPLE_TRANSLATION;
        b.compound_type = COMPOUND_AVERAGE;
        b.pal_y = b.pal_uv = 0;
        b.interp[0] = b.interp[1] = BILINEAR;
        MvStack s;
        find_mv_stack(b, s);
        assign_mv(b, s, false);
    } else {
        b.is_inter = false;
        const int above = b.avail_u ? mi(b.r - 1, b.c).y_mode : DC_PRED;
        const int left = b.avail_l ? mi(b.r, b.c - 1).y_mode : DC_PRED;
        b.y_mode = S(cdf.mode.kf_y[kIntraModeContext[above]][kIntraModeContext[left]], 13);
        intra_angle_info_y(b);
        if (b.has_chroma) read_uv_mode(b);
        b.pal_y = b.pal_uv = 0;
        if (b.bsize >= BLOCK_8X8 && b.bw4 <= 16 && b.bh4 <= 16 && fh.allow_screen_content_tools) palette_mode_info(b);
        filter_intra_mode_info(b);
    }
}

// intra_block_mode_info (Block.cpp:1390-1412)
void BlockParser::intra_block_mode_info(Blk& b)
{
    b.ref[0] = INTRA_FRAME;
    b.ref[1] = NONE_FRAME;
    b.y_mode = S(cdf.mode.y_mode[kSizeGroup[b.bsize]], 13);
    intra_angle_info_y(b);
    if (b.has_chroma) read_uv_mode(b);
    b.pal_y = b.pal_uv = 0;
    if (b.bsize >= BLOCK_8X8 && b.bw4 <= 16 && b.bh4 <= 16 && fh.allow_screen_content_tools) palette_mode_info(b);
    filter_intra_mode_info(b);
}

// inter_frame_mode_info (Block.cpp:1414-1448)
void BlockParser::inter_frame_mode_info(Blk& b)
{
    b.use_intrabc = false;
    b.left_ref[0] = b.avail_l ? mi(b.r, b.c - 1).ref[0] : INTRA_FRAME;
    b.above_ref[0] = b.avail_u ? mi(b.r - 1, b.c).ref[0] : INTRA_FRAME;
    b.left_ref[1] = b.avail_l ? mi(b.r, b.c - 1).ref[1] : NONE_FRAME;
    b.above_ref[1] = b.avail_u ? mi(b.r - 1, b.c).ref[1] : NONE_FRAME;
    b.left_intra = b.left_ref[0] <= INTRA_FRAME;
    b.above_intra = b.above_ref[0] <= INTRA_FRAME;
    b.left_single = b.left_ref[1] <= INTRA_FRAME;
    b.above_single = b.above_ref[1] <= INTRA_FRAME;
    b.skip = false;
    // read_skip_mode (Block.cpp:625-639)
    if (!fh.skip_mode_present || bw4_of(b.bsize) < 2 || bh4_of(b.bsize) < 2) {
        b.skip_mode = false;
    } else {
        int ctx = 0;
        if (b.avail_u) ctx += mi(b.r - 1, b.c).skip_mode;
        if (b.avail_l) ctx += mi(b.r, b.c - 1).skip_mode;
        b.skip_mode = S(cdf.mode.skip_mode[ctx], 2) != 0;
    }
    b.skip = b.skip_mode ? true : read_skip(b);
    b.lossless = fh.coded_lossless;
    read_cdef(b);
    read_delta_qindex(b);
    read_delta_lf(b);
    T.read_deltas = false;
    // read_is_inter (Block.cpp:641-665)
    if (b.skip_mode) {
        b.is_inter = true;
    } else {
        int ctx;
        if (b.avail_u && b.avail_l) ctx = (b.left_intra && b.above_intra) ? 3 : (b.left_intra || b.above_intra);
        else if (b.avail_u || b.avail_l) ctx = 2 * (b.avail_u ? b.above_intra : b.left_intra);
        else ctx = 0;
        b.is_inter = S(cdf.mode.intra_inter[ctx], 2) != 0;
    }
    if (b.is_inter) inter_block_mode_info(b);
    else intra_block_mode_info(b);
}

// ------------------------------------------------------------------------------------
// reference frames (Block.cpp:1618-1936)
// ------------------------------------------------------------------------------------
int BlockParser::count_refs(const Blk& b, int type) const
{
    int n = 0;
    if (b.avail_u) n += (b.above_ref[0] == type) + (b.above_ref[1] == type);
    if (b.avail_l) n += (b.left_ref[0] == type) + (b.left_ref[1] == type);
    return n;
}
static int ref_count_ctx(int c0, int c1) { return c0 < c1 ? 0 : c0 == c1 ? 1 : 2; }
static bool check_backward(int ref) { return ref >= BWDREF_FRAME && ref <= ALTREF_FRAME; }

void BlockParser::read_ref_frames(Blk& b)
{
    if (b.skip_mode) {
        b.ref[0] = fh.skip_mode_frame[0];
        b.ref[1] = fh.skip_mode_frame[1];
        return;
    }
    bool compound = false;
    if (fh.reference_select && std::min(b.bw4, b.bh4) >= 2) {
        int ctx;
        if (b.avail_u && b.avail_l) {
            if (b.above_single && b.left_single) ctx = check_backward(b.above_ref[0]) ^ check_backward(b.left_ref[0]);
            else if (b.above_single) ctx = 2 + (check_backward(b.above_ref[0]) || b.above_intra);
            else if (b.left_single) ctx = 2 + (check_backward(b.left_ref[0]) || b.left_intra);
            else ctx = 4;
        } else if (b.avail_u) {
            ctx = b.above_single ? check_backward(b.above_ref[0]) : 3;
        } else if (b.avail_l) {
            ctx = b.left_single ? check_backward(b.left_ref[0]) : 3;
        } else {
            ctx = 1;
        }
        compound = S(cdf.mode.comp_inter[ctx], 2) != 0;
    }
    if (compound) read_comp_reference(b);
    else read_single_reference(b);
}

void BlockParser::read_comp_reference(Blk& b)
{
    // comp_ref_type context (Block.cpp:1697-1745), operands as uint8 like the reference
    const uint8_t above0 = (uint8_t)b.above_ref[0], above1 = (uint8_t)b.above_ref[1];
    const uint8_t left0 = (uint8_t)b.left_ref[0], left1 = (uint8_t)b.left_ref[1];
    auto samedir = [](uint8_t a, uint8_t c) { return (a >= BWDREF_FRAME) == (c >= BWDREF_FRAME); };
    const bool aboveComp = b.avail_u && !b.above_intra && !b.above_single;
    const bool leftComp = b.avail_l && !b.left_intra && !b.left_single;
    const bool aboveUni = aboveComp && samedir(above0, above1);
    const bool leftUni = leftComp && samedir(left0, left1);
    int ctx;
    if (b.avail_u && !b.above_intra && b.avail_l && !b.left_intra) {
        const bool sd2 = samedir(above0, left0);
        if (!aboveComp && !leftComp) ctx = 1 + 2 * sd2;
        else if (!aboveComp) ctx = !leftUni ? 1 : 3 + sd2;
        else if (!leftComp) ctx = !aboveUni ? 1 : 3 + sd2;
        else if (!aboveUni && !leftUni) ctx = 0;
        else if (!aboveUni || !leftUni) ctx = 2;
        else ctx = 3 + ((above0 == BWDREF_FRAME) == (left0 == BWDREF_FRAME));
    } else if (b.avail_u && b.avail_l) {
        if (aboveComp) ctx = 1 + 2 * aboveUni;
        else if (leftComp) ctx = 1 + 2 * leftUni;
        else ctx = 2;
    } else if (aboveComp) {
        ctx = 4 * aboveUni;
    } else if (leftComp) {
        ctx = 4 * leftUni;
    } else {
        ctx = 2;
    }
    const int fwd = count_refs(b, LAST_FRAME) + count_refs(b, LAST2_FRAME) + count_refs(b, LAST3_FRAME) + count_refs(b, GOLDEN_FRAME);
    const int bwd = count_refs(b, BWDREF_FRAME) + count_refs(b, ALTREF2_FRAME) + count_refs(b, ALTREF_FRAME);
    const int ctxP1 = ref_count_ctx(fwd, bwd);
    const int ctxL12 = ref_count_ctx(count_refs(b, LAST_FRAME) + count_refs(b, LAST2_FRAME),
                                     count_refs(b, LAST3_FRAME) + count_refs(b, GOLDEN_FRAME));
    const int ctxL1 = ref_count_ctx(count_refs(b, LAST_FRAME), count_refs(b, LAST2_FRAME));
    const int ctxL3G = ref_count_ctx(count_refs(b, LAST3_FRAME), count_refs(b, GOLDEN_FRAME));
    const int ctxBwd = ref_count_ctx(count_refs(b, BWDREF_FRAME) + count_refs(b, ALTREF2_FRAME), count_refs(b, ALTREF_FRAME));
    const int ctxBwdP1 = ref_count_ctx(count_refs(b, BWDREF_FRAME), count_refs(b, ALTREF2_FRAME));
    const int type = S(cdf.mode.comp_ref_type[ctx], 2);
    if (type == 0) {  // UNIDIR_COMP_REFERENCE
        if (S(cdf.mode.uni_comp_ref[ctxP1][0], 2)) {
            b.ref[0] = BWDREF_FRAME;
            b.ref[1] = ALTREF_FRAME;
        } else {
            const int ctxU1 = ref_count_ctx(count_refs(b, LAST2_FRAME), count_refs(b, LAST3_FRAME) + count_refs(b, GOLDEN_FRAME));
            if (S(cdf.mode.uni_comp_ref[ctxU1][1], 2)) {
                b.ref[0] = LAST_FRAME;
                b.ref[1] = S(cdf.mode.uni_comp_ref[ctxL3G][2], 2) ? GOLDEN_FRAME : LAST3_FRAME;
            } else {
                b.ref[0] = LAST_FRAME;
                b.ref[1] = LAST2_FRAME;
            }
        }
    } else {
        if (!S(cdf.mode.comp_ref[ctxL12][0], 2)) b.ref[0] = S(cdf.mode.comp_ref[ctxL1][1], 2) ? LAST2_FRAME : LAST_FRAME;
        else b.ref[0] = S(cdf.mode.comp_ref[ctxL3G][2], 2) ? GOLDEN_FRAME : LAST3_FRAME;
        if (!S(cdf.mode.comp_bwdref[ctxBwd][0], 2)) b.ref[1] = S(cdf.mode.comp_bwdref[ctxBwdP1][1], 2) ? ALTREF2_FRAME : BWDREF_FRAME;
        else b.ref[1] = ALTREF_FRAME;
    }
}

void BlockParser::read_single_reference(Blk& b)
{
    const int fwd = count_refs(b, LAST_FRAME) + count_refs(b, LAST2_FRAME) + count_refs(b, LAST3_FRAME) + count_refs(b, GOLDEN_FRAME);
    const int bwd = count_refs(b, BWDREF_FRAME) + count_refs(b, ALTREF2_FRAME) + count_refs(b, ALTREF_FRAME);
    if (S(cdf.mode.single_ref[ref_count_ctx(fwd, bwd)][0], 2)) {
        const int c2 = ref_count_ctx(count_refs(b, BWDREF_FRAME) + count_refs(b, ALTREF2_FRAME), count_refs(b, ALTREF_FRAME));
        if (!S(cdf.mode.single_ref[c2][1], 2)) {
            const int c6 = ref_count_ctx(count_refs(b, BWDREF_FRAME), count_refs(b, ALTREF2_FRAME));
            b.ref[0] = S(cdf.mode.single_ref[c6][5], 2) ? ALTREF2_FRAME : BWDREF_FRAME;
        } else {
            b.ref[0] = ALTREF_FRAME;
        }
    } else {
        const int c3 = ref_count_ctx(count_refs(b, LAST_FRAME) + count_refs(b, LAST2_FRAME),
                                     count_refs(b, LAST3_FRAME) + count_refs(b, GOLDEN_FRAME));
        if (S(cdf.mode.single_ref[c3][2], 2)) {
            const int c5 = ref_count_ctx(count_refs(b, LAST3_FRAME), count_refs(b, GOLDEN_FRAME));
            b.ref[0] = S(cdf.mode.single_ref[c5][4], 2) ? GOLDEN_FRAME : LAST3_FRAME;
        } else {
            const int c4 = ref_count_ctx(count_refs(b, LAST_FRAME), count_refs(b, LAST2_FRAME));
            b.ref[0] = S(cdf.mode.single_ref[c4][3], 2) ? LAST2_FRAME : LAST_FRAME;
        }
    }
    b.ref[1] = NONE_FRAME;
}

// ------------------------------------------------------------------------------------
// inter block mode info (Block.cpp:760-841, 887-927, 1202-1388)
// ------------------------------------------------------------------------------------
static bool has_newmv(int mode)
{
    return mode == NEWMV || mode == NEW_NEWMV || mode == NEAR_NEWMV || mode == NEW_NEARMV || mode == NEAREST_NEWMV ||
           mode == NEW_NEARESTMV;
}

void BlockParser::inter_block_mode_info(Blk& b)
{
    b.pal_y = b.pal_uv = 0;
    read_ref_frames(b);
    const bool isCompound = b.ref[1] > INTRA_FRAME;
    MvStack s;
    find_mv_stack(b, s);
    if (b.skip_mode) {
        b.y_mode = NEAREST_NEARESTMV;
    } else if (isCompound) {
        const int ctx = kCompoundModeCtxMap[s.ref_ctx >> 1][std::min(s.new_ctx, 4)];
        b.y_mode = NEAREST_NEARESTMV + S(cdf.mode.inter_compound_mode[ctx], 8);
    } else {
        if (!S(cdf.mode.newmv[s.new_ctx], 2)) {
            b.y_mode = NEWMV;
        } else if (!S(cdf.mode.zeromv[s.zero_ctx], 2)) {
            b.y_mode = GLOBALMV;
        } else {
            b.y_mode = !S(cdf.mode.refmv[s.ref_ctx], 2) ? NEARESTMV : NEARMV;
        }
    }
    b.ref_mv_idx = 0;
    if (b.y_mode == NEWMV || b.y_mode == NEW_NEWMV) {
        for (int idx = 0; idx < 2; idx++)
            if (s.num > idx + 1) {
                if (!S(cdf.mode.drl[s.drl_ctx[idx]], 2)) {
                    b.ref_mv_idx = idx;
                    break;
                }
                b.ref_mv_idx = idx + 1;
            }
    } else if (b.y_mode == NEARMV || b.y_mode == NEAR_NEARMV || b.y_mode == NEAR_NEWMV || b.y_mode == NEW_NEARMV) {
        b.ref_mv_idx = 1;
        for (int idx = 1; idx < 3; idx++)
            if (s.num > idx + 1) {
                if (!S(cdf.mode.drl[s.drl_ctx[idx]], 2)) {
                    b.ref_mv_idx = idx;
                    break;
                }
                b.ref_mv_idx = idx + 1;
            }
    }
    assign_mv(b, s, isCompound);
    read_interintra_mode(b, isCompound);
    read_motion_mode(b, isCompound);
    read_compound_type(b, isCompound);
    if (fh.interpolation_filter == SWITCHABLE) {
        for (int dir = 0; dir < (seq.enable_dual_filter ? 2 : 1); dir++)
            b.interp[dir] = needs_interp_filter(b) ? S(cdf.mode.switchable_interp[interp_filter_ctx(b, dir)], 3) : EIGHTTAP;
        if (!seq.enable_dual_filter) b.interp[1] = b.interp[0];
    } else {
        b.interp[0] = b.interp[1] = fh.interpolation_filter;
    }
}

bool BlockParser::needs_interp_filter(const Blk& b) const
{
    const bool large = std::min(b.bw4, b.bh4) >= 2;
    if (b.skip_mode || b.motion_mode == LOCALWARP) return false;
    if (large && b.y_mode == GLOBALMV) return fh.gm_type[b.ref[0]] == GM_TRANSLATION;
    if (large && b.y_mode == GLOBAL_GLOBALMV)
        return fh.gm_type[b.ref[0]] == GM_TRANSLATION || fh.gm_type[b.ref[1]] == GM_TRANSLATION;
    return true;
}

int BlockParser::interp_filter_ctx(const Blk& b, int dir)
{
    int ctx = ((dir & 1) * 2 + (b.ref[1] > INTRA_FRAME)) * 4;
    int leftType = 3, aboveType = 3;
    if (b.avail_l) {
        const MiInfo& m = mi(b.r, b.c - 1);
        if (m.ref[0] == b.ref[0] || m.ref[1] == b.ref[0]) leftType = m.interp[dir];
    }
    if (b.avail_u) {
        const MiInfo& m = mi(b.r - 1, b.c);
        if (m.ref[0] == b.ref[0] || m.ref[1] == b.ref[0]) aboveType = m.interp[dir];
    }
    if (leftType == aboveType) ctx += leftType;
    else if (leftType == 3) ctx += aboveType;
    else if (aboveType == 3) ctx += leftType;
    else ctx += 3;
    return ctx;
}

bool BlockParser::is_scaled(int refFrame) const  // FrameHeader::is_scaled (Parser.cpp:788-803)
{
    const RefSlot& r = P.slots[fh.ref_frame_idx[refFrame - LAST_FRAME]];
    const uint32_t xs = (((uint32_t)r.upscaled_width << 14) + (fh.frame_width / 2)) / fh.frame_width;
    const uint32_t ys = (((uint32_t)r.frame_height << 14) + (fh.frame_height / 2)) / fh.frame_height;
    return xs != (1u << 14) || ys != (1u << 14);
}

void BlockParser::read_compound_type(Blk& b, bool isCompound)
{
    b.comp_group_idx = false;
    b.compound_idx = true;
    if (b.skip_mode) {
        b.compound_type = COMPOUND_AVERAGE;
        return;
    }
    if (isCompound) {
        const int n = av1r_wedge_bits[b.bsize];
        if (seq.enable_masked_compound) {
            int ctx = 0;
            if (b.avail_u) {
                if (!b.above_single) ctx += mi(b.r - 1, b.c).comp_group_idx;
                else if (b.above_ref[0] == ALTREF_FRAME) ctx += 3;
            }
            if (b.avail_l) {
                if (!b.left_single) ctx += mi(b.r, b.c - 1).comp_group_idx;
                else if (b.left_ref[0] == ALTREF_FRAME) ctx += 3;
            }
            b.comp_group_idx = S(cdf.mode.comp_group_idx[std::min(5, ctx)], 2) != 0;
        }
        if (!b.comp_group_idx) {
            if (seq.enable_jnt_comp) {
                const int fwd = abs(P.relative_dist(fh.order_hints[b.ref[0]], fh.order_hint));
                const int bck = abs(P.relative_dist(fh.order_hints[b.ref[1]], fh.order_hint));
                int ctx = (fwd == bck) ? 3 : 0;
                if (b.avail_u) {
                    if (!b.above_single) ctx += mi(b.r - 1, b.c).compound_idx;
                    else if (b.above_ref[0] == ALTREF_FRAME) ctx++;
                }
                if (b.avail_l) {
                    if (!b.left_single) ctx += mi(b.r, b.c - 1).compound_idx;
                    else if (b.left_ref[0] == ALTREF_FRAME) ctx++;
                }
                b.compound_idx = S(cdf.mode.compound_index[ctx], 2) != 0;
                b.compound_type = b.compound_idx ? COMPOUND_AVERAGE : COMPOUND_DISTANCE;
            } else {
                b.compound_type = COMPOUND_AVERAGE;
            }
        } else {
            b.compound_type = n == 0 ? COMPOUND_DIFFWTD : S(cdf.mode.compound_type[b.bsize], 2);
        }
        if (b.compound_type == COMPOUND_WEDGE) {
            b.wedge_index = S(cdf.mode.wedge_idx[b.bsize], 16);
            b.wedge_sign = sd.boolean();
        } else if (b.compound_type == COMPOUND_DIFFWTD) {
            b.mask_type = sd.boolean() != 0;
        }
    } else {
        b.compound_type = b.interintra ? (b.wedge_interintra ? COMPOUND_WEDGE : COMPOUND_INTRA) : COMPOUND_AVERAGE;
    }
}

bool BlockParser::has_overlappable_candidates(const Blk& b)
{
    if (b.avail_u)
        for (int x4 = b.c; x4 < std::min(fh.mi_cols, b.c + b.bw4); x4 += 2)
            if (mi(b.r - 1, x4 | 1).ref[0] > INTRA_FRAME) return true;
    if (b.avail_l)
        for (int y4 = b.r; y4 < std::min(fh.mi_rows, b.r + b.bh4); y4 += 2)
            if (mi(y4 | 1, b.c - 1).ref[0] > INTRA_FRAME) return true;
    return false;
}

void BlockParser::read_motion_mode(Blk& b, bool isCompound)
{
    b.motion_mode = SIMPLE_TRANSLATION;
    if (b.skip_mode || !fh.is_motion_mode_switchable) return;
    if (std::min(b.bw4, b.bh4) < 2) return;
    if (!fh.force_integer_mv && (b.y_mode == GLOBALMV || b.y_mode == GLOBAL_GLOBALMV) && fh.gm_type[b.ref[0]] > GM_TRANSLATION)
        return;
    if (isCompound || b.ref[1] == INTRA_FRAME || !has_overlappable_candidates(b)) return;
    find_warp_samples(b);
    if (fh.force_integer_mv || b.num_samples == 0 || !fh.allow_warped_motion || is_scaled(b.ref[0]))
        b.motion_mode = S(cdf.mode.obmc[b.bsize], 2) ? OBMC_CAUSAL : SIMPLE_TRANSLATION;
    else
        b.motion_mode = S(cdf.mode.motion_mode[b.bsize], 3);
}

void BlockParser::read_interintra_mode(Blk& b, bool isCompound)
{
    b.interintra = false;
    if (!b.skip_mode && seq.enable_interintra_compound && !isCompound && b.bsize >= BLOCK_8X8 && b.bsize <= BLOCK_32X32) {
        b.interintra = S(cdf.mode.interintra[kSizeGroup[b.bsize]], 2) != 0;
        if (b.interintra) {
            b.interintra_mode = S(cdf.mode.interintra_mode[kSizeGroup[b.bsize]], 4);
            b.ref[1] = INTRA_FRAME;
            b.angle_y = b.angle_uv = 0;
            b.use_filter_intra = false;
            b.wedge_interintra = S(cdf.mode.wedge_interintra[b.bsize], 2) != 0;
            if (b.wedge_interintra) {
                b.wedge_index = S(cdf.mode.wedge_idx[b.bsize], 16);
                b.wedge_sign = 0;
            }
        }
    }
}

int BlockParser::read_mv_component(int ctx, int comp)
{
    MvComp& m = cdf.mv[ctx].comp[comp];
    const bool sign = S(m.sign, 2) != 0;
    const int cls = S(m.classes, 11);
    int mag;
    if (cls == 0) {
        const int bit = S(m.class0, 2);
        const int fr = fh.force_integer_mv ? 3 : S(m.class0_fp[bit], 4);
        const int hp = fh.allow_high_precision_mv ? S(m.class0_hp, 2) : 1;
        mag = ((bit << 3) | (fr << 1) | hp) + 1;
    } else {
        int d = 0;
        for (int i = 0; i < cls; i++) d |= S(m.bits[i], 2) << i;
        mag = 2 << (cls + 2);  // CLASS0_SIZE << (mv_class + 2)
        const int fr = fh.force_integer_mv ? 3 : S(m.fp, 4);
        const int hp = fh.allow_high_precision_mv ? S(m.hp, 2) : 1;
        mag += ((d << 3) | (fr << 1) | hp) + 1;
    }
    return sign ? -mag : mag;
}

void BlockParser::read_mv(Blk& b, const Mv* pred, int ref)
{
    const int ctx = b.use_intrabc ? 1 : 0;
    int diff[2] = {0, 0};
#ifdef AV1P_WRITER
    if (sd.hook) sd.hook->mv_pred(pred[ref], ctx);
#endif
    const int joint = S(cdf.mv[ctx].joints, 4);
    if (joint == 2 || joint == 3) diff[0] = read_mv_component(ctx, 0);
    if (joint == 1 || joint == 3) diff[1] = read_mv_component(ctx, 1);
    b.mv[ref].r = (int16_t)(pred[ref].r + diff[0]);
    b.mv[ref].c = (int16_t)(pred[ref].c + diff[1]);
}

static int comp_mode_of(int yMode, int refList)  // Block::get_mode (Block.cpp:1259-1284)
{
    if (refList == 0) {
        if (yMode < NEAREST_NEARESTMV) return yMode;
        if (yMode == NEW_NEWMV || yMode == NEW_NEARESTMV || yMode == NEW_NEARMV) return NEWMV;
        if (yMode == NEAREST_NEARESTMV || yMode == NEAREST_NEWMV) return NEARESTMV;
        if (yMode == NEAR_NEARMV || yMode == NEAR_NEWMV) return NEARMV;
        return GLOBALMV;
    }
    if (yMode == NEW_NEWMV || yMode == NEAREST_NEWMV || yMode == NEAR_NEWMV) return NEWMV;
    if (yMode == NEAREST_NEARESTMV || yMode == NEW_NEARESTMV) return NEARESTMV;
    if (yMode == NEAR_NEARMV || yMode == NEW_NEARMV) return NEARMV;
    return GLOBALMV;
}

void BlockParser::assign_mv(Blk& b, const MvStack& s, bool isCompound)
{
    Mv pred[2];
    for (int i = 0; i < 1 + isCompound; i++) {
        const int compMode = b.use_intrabc ? NEWMV : comp_mode_of(b.y_mode, i);
        if (b.use_intrabc) {
            pred[0] = s.stack[0][0];
            if (pred[0].r == 0 && pred[0].c == 0) pred[0] = s.stack[1][0];
            if (pred[0].r == 0 && pred[0].c == 0) {
                const int sbSize4 = seq.use_128x128 ? 32 : 16;
                if (b.r - sbSize4 < T.mi_row_start) {
                    pred[0].r = 0;
                    pred[0].c = (int16_t)(-(sbSize4 * 4 + 256) * 8);
                } else {
                    pred[0].r = (int16_t)(-(sbSize4 * 4 * 8));
                    pred[0].c = 0;
                }
            }
        } else if (compMode == GLOBALMV) {
            pred[i] = s.global[i];
        } else {
            int pos = compMode == NEARESTMV ? 0 : b.ref_mv_idx;
            if (compMode == NEWMV && s.num <= 1) pos = 0;
            pred[i] = s.stack[pos][i];
        }
        if (compMode == NEWMV) read_mv(b, pred, i);
        else b.mv[i] = pred[i];
    }
}

// ------------------------------------------------------------------------------------
// FindMvStack (InterPredict.cpp:1051-1669)
// ------------------------------------------------------------------------------------
void BlockParser::lower_mv_precision(Mv& mv) const
{
    if (fh.allow_high_precision_mv) return;
    int16_t* v[2] = {&mv.r, &mv.c};
    for (int i = 0; i < 2; i++) {
        int16_t& x = *v[i];
        if (fh.force_integer_mv) {
            const int a = abs(x);
            const int aInt = (a + 3) >> 3;
            x = (int16_t)(x > 0 ? (aInt << 3) : -(aInt << 3));
        } else if (x & 1) {
            x = (int16_t)(x > 0 ? x - 1 : x + 1);
        }
    }
}

void BlockParser::setup_global_mv(const Blk& b, MvStack& s, int refList)
{
    Mv& mv = s.global[refList];
    const int ref = (uint8_t)b.ref[refList];
    const int typ = ref != INTRA_FRAME ? fh.gm_type[ref] : GM_IDENTITY;
    if (ref == INTRA_FRAME || typ == GM_IDENTITY) {
        mv.r = mv.c = 0;
    } else if (typ == GM_TRANSLATION) {
        mv.r = (int16_t)(fh.gm_params[ref][0] >> (kWarpPrecBits - 3));
        mv.c = (int16_t)(fh.gm_params[ref][1] >> (kWarpPrecBits - 3));
    } else {
        const int x = b.c * 4 + b.bw4 * 2 - 1;
        const int y = b.r * 4 + b.bh4 * 2 - 1;
        const int32_t* g = fh.gm_params[ref];
        const int xc = (g[2] - (1 << kWarpPrecBits)) * x + g[3] * y + g[0];
        const int yc = g[4] * x + (g[5] - (1 << kWarpPrecBits)) * y + g[1];
        if (fh.allow_high_precision_mv) {
            mv.r = (int16_t)round2signed_64(yc, kWarpPrecBits - 3);
            mv.c = (int16_t)round2signed_64(xc, kWarpPrecBits - 3);
        } else {
            mv.r = (int16_t)(round2signed_64(yc, kWarpPrecBits - 2) * 2);
            mv.c = (int16_t)(round2signed_64(xc, kWarpPrecBits - 2) * 2);
        }
    }
    lower_mv_precision(mv);
}

void BlockParser::search_stack(const Blk& b, MvStack& s, int mvRow, int mvCol, int candList, uint32_t weight)
{
    const MiInfo& m = mi(mvRow, mvCol);
    const int candMode = m.y_mode;
    const int candSize = m.mi_size;
    const bool large = std::min(bw4_of(candSize), bh4_of(candSize)) >= 2;
    Mv cand;
    if ((candMode == GLOBALMV || candMode == GLOBAL_GLOBALMV) && fh.gm_type[b.ref[0]] > GM_TRANSLATION && large)
        cand = s.global[0];
    else
        cand = m.mv[candList];
    lower_mv_precision(cand);
    if (has_newmv(candMode)) s.new_count++;
    s.found = true;
    int idx;
    for (idx = 0; idx < s.num; idx++)
        if (cand == s.stack[idx][0]) break;
    if (idx < s.num) {
        s.weight[idx] += weight;
    } else if (idx < kMaxRefMvStack) {
        s.stack[s.num][0] = cand;
        s.weight[s.num] = weight;
        s.num++;
    }
}

void BlockParser::search_compound_stack(const Blk& b, MvStack& s, int mvRow, int mvCol, uint32_t weight)
{
    const MiInfo& m = mi(mvRow, mvCol);
    Mv cand[2] = {m.mv[0], m.mv[1]};
    const int candMode = m.y_mode;
    if (candMode == GLOBAL_GLOBALMV)
        for (int i = 0; i < 2; i++)
            if (fh.gm_type[b.ref[i]] > GM_TRANSLATION) cand[i] = s.global[i];
    lower_mv_precision(cand[0]);
    lower_mv_precision(cand[1]);
    if (has_newmv(candMode)) s.new_count++;
    s.found = true;
    int idx;
    for (idx = 0; idx < s.num; idx++)
        if (cand[0] == s.stack[idx][0] && cand[1] == s.stack[idx][1]) break;
    if (idx < s.num) {
        s.weight[idx] += weight;
    } else if (idx < kMaxRefMvStack) {
        s.stack[s.num][0] = cand[0];
        s.stack[s.num][1] = cand[1];
        s.weight[s.num] = weight;
        s.num++;
    }
}

void BlockParser::add_ref_mv_candidate(const Blk& b, MvStack& s, int mvRow, int mvCol, uint32_t weight)
{
    const MiInfo& m = mi(mvRow, mvCol);
    if (!m.is_inter) return;
    const bool isCompound = b.ref[1] > INTRA_FRAME;
    if (!isCompound) {
        for (int candList = 0; candList < 2; candList++)
            if (m.ref[candList] == b.ref[0]) search_stack(b, s, mvRow, mvCol, candList, weight);
    } else if (m.ref[0] == b.ref[0] && m.ref[1] == b.ref[1]) {
        search_compound_stack(b, s, mvRow, mvCol, weight);
    }
}

void BlockParser::scan_row(const Blk& b, MvStack& s, int deltaRow)
{
    int deltaCol = 0;
    const int end4 = std::min(std::min(b.bw4, fh.mi_cols - b.c), 16);
    const bool useStep16 = b.bw4 >= 16;
    if (abs(deltaRow) > 1) {
        deltaRow += b.r & 1;
        deltaCol = 1 - (b.c & 1);
    }
    int i = 0;
    while (i < end4) {
        const int mvRow = b.r + deltaRow, mvCol = b.c + deltaCol + i;
        if (!inside(mvRow, mvCol)) break;
        int len = std::min(b.bw4, bw4_of(mi(mvRow, mvCol).mi_size));
        if (abs(deltaRow) > 1) len = std::max(2, len);
        if (useStep16) len = std::max(4, len);
        add_ref_mv_candidate(b, s, mvRow, mvCol, (uint32_t)len * 2);
        i += len;
    }
}

void BlockParser::scan_col(const Blk& b, MvStack& s, int deltaCol)
{
    int deltaRow = 0;
    const int end4 = std::min(std::min(b.bh4, fh.mi_rows - b.r), 16);
    const bool useStep16 = b.bh4 >= 16;
    if (abs(deltaCol) > 1) {
        deltaRow = 1 - (b.r & 1);
        deltaCol += b.c & 1;
    }
    int i = 0;
    while (i < end4) {
        const int mvRow = b.r + deltaRow + i, mvCol = b.c + deltaCol;
        if (!inside(mvRow, mvCol)) break;
        int len = std::min(b.bh4, bh4_of(mi(mvRow, mvCol).mi_size));
        if (abs(deltaCol) > 1) len = std::max(2, len);
        if (useStep16) len = std::max(4, len);
        add_ref_mv_candidate(b, s, mvRow, mvCol, (uint32_t)len * 2);
        i += len;
    }
}

void BlockParser::scan_point(const Blk& b, MvStack& s, int deltaRow, int deltaCol)
{
    const int mvRow = b.r + deltaRow, mvCol = b.c + deltaCol;
    // positions not yet decoded hold zeroed mode info (not inter): add_ref_mv_candidate
    // ignores them, as the reference's RefFrames[0] != NONE_FRAME test does
    if (inside(mvRow, mvCol)) add_ref_mv_candidate(b, s, mvRow, mvCol, 4);
}

// add_tpl_ref_mv (InterPredict.cpp:1051-1126) for every position of temporalScan
// (InterPredict.cpp:1128-1153), with the block's invariants hoisted (the reference lists'
// motion fields, the compound test) and the last stack entry a position matched (neighbouring positions mostly project the
// same motion vector; the stack holds distinct entries, so a match there is the match the
// spec's linear search finds)
void BlockParser::temporal_scan(const Blk& b, MvStack& s)
{
    const int stepW4 = b.bw4 >= 16 ? 4 : 2, stepH4 = b.bh4 >= 16 ? 4 : 2;
    const bool isCompound = b.ref[1] > INTRA_FRAME;
    const Mv* mf0 = P.motion_field[b.ref[0]].data();
    const Mv* mf1 = isCompound ? P.motion_field[b.ref[1]].data() : nullptr;
    const size_t stride8 = (size_t)(fh.aligned_mi_cols >> 1);
    int last = -1;
    auto add = [&](int deltaRow, int deltaCol) {
        const int mvRow = (b.r + deltaRow) | 1, mvCol = (b.c + deltaCol) | 1;
        if (!inside(mvRow, mvCol)) return;
        const size_t at = (size_t)(mvRow >> 1) * stride8 + (mvCol >> 1);
        const bool origin = deltaRow == 0 && deltaCol == 0;
        if (origin) s.zero_ctx = 1;
        Mv c0 = mf0[at];
        if (c0.r == (int16_t)INT16_MIN) return;
        Mv c1 = {0, 0};
        if (isCompound) {
            c1 = mf1[at];
            if (c1.r == (int16_t)INT16_MIN) return;
            lower_mv_precision(c1);
        }
        lower_mv_precision(c0);
        if (origin)
            s.zero_ctx = (abs(c0.r - s.global[0].r) >= 16 || abs(c0.c - s.global[0].c) >= 16 ||
                          (isCompound && (abs(c1.r - s.global[1].r) >= 16 || abs(c1.c - s.global[1].c) >= 16)))
                             ? 1
                             : 0;
        auto same = [&](int idx) { return c0 == s.stack[idx][0] && (!isCompound || c1 == s.stack[idx][1]); };
        int idx = -1;
        if (last >= 0 && same(last)) {
            idx = last;
        } else {
            for (int i = 0; i < s.num; i++)
                if (same(i)) {
                    idx = i;
                    break;
                }
        }
        if (idx >= 0) {
            s.weight[idx] += 2;
            last = idx;
        } else if (s.num < kMaxRefMvStack) {
            s.stack[s.num][0] = c0;
            if (isCompound) s.stack[s.num][1] = c1;
            s.weight[s.num] = 2;
            last = s.num++;
        }
    };
    for (int dr = 0; dr < std::min(b.bh4, 16); dr += stepH4)
        for (int dc = 0; dc < std::min(b.bw4, 16); dc += stepW4) add(dr, dc);
    const bool allowExtension = b.bh4 >= 2 && b.bh4 < 16 && b.bw4 >= 2 && b.bw4 < 16;
    if (allowExtension) {
        const int pos[3][2] = {{b.bh4, -2}, {b.bh4, b.bw4}, {b.bh4 - 2, b.bw4}};
        for (auto& p : pos) {
            const int row = (b.r & 15) + p[0], col = (b.c & 15) + p[1];
            if (row >= 0 && row < 16 && col >= 0 && col < 16) add(p[0], p[1]);
        }
    }
}

void BlockParser::add_extra_mv_candidate(const Blk& b, MvStack& s, int mvRow, int mvCol, MvList2* idMvs,
                                         MvList2* diffMvs)
{
    const MiInfo& m = mi(mvRow, mvCol);
    if (b.ref[1] > INTRA_FRAME) {
        for (int candList = 0; candList < 2; candList++) {
            const int candRef = m.ref[candList];
            if (candRef <= INTRA_FRAME) continue;
            for (int list = 0; list < 2; list++) {
                Mv cand = m.mv[candList];
                if (candRef == b.ref[list] && idMvs[list].size() < 2) {
                    idMvs[list].push_back(cand);
                } else if (diffMvs[list].size() < 2) {
                    if (fh.ref_frame_sign_bias[candRef] != fh.ref_frame_sign_bias[b.ref[list]]) {
                        cand.r = (int16_t)(cand.r * -1);
                        cand.c = (int16_t)(cand.c * -1);
                    }
                    diffMvs[list].push_back(cand);
                }
            }
        }
    } else {
        for (int candList = 0; candList < 2; candList++) {
            const int candRef = m.ref[candList];
            if (candRef <= INTRA_FRAME) continue;
            Mv cand = m.mv[candList];
            if (fh.ref_frame_sign_bias[candRef] != fh.ref_frame_sign_bias[b.ref[0]]) {
                cand.r = (int16_t)(cand.r * -1);
                cand.c = (int16_t)(cand.c * -1);
            }
            int idx;
            for (idx = 0; idx < s.num; idx++)
                if (cand == s.stack[idx][0]) break;
            if (idx == s.num) {
                s.stack[idx][0] = cand;
                s.weight[idx] = 2;
                s.num++;
            }
        }
    }
}

void BlockParser::extra_search(const Blk& b, MvStack& s)
{
    MvList2 idMvs[2], diffMvs[2];  // at most 2 each (the spec's idMvs / diffMvs)
    int w4 = std::min(16, b.bw4), h4 = std::min(16, b.bh4);
    w4 = std::min(w4, fh.mi_cols - b.c);
    h4 = std::min(h4, fh.mi_rows - b.r);
    const int num4x4 = std::min(w4, h4);
    for (int pass = 0; pass < 2; pass++) {
        int idx = 0;
        while (idx < num4x4 && s.num < 2) {
            const int mvRow = pass == 0 ? b.r - 1 : b.r + idx;
            const int mvCol = pass == 0 ? b.c + idx : b.c - 1;
            if (!inside(mvRow, mvCol)) break;
            add_extra_mv_candidate(b, s, mvRow, mvCol, idMvs, diffMvs);
            idx += pass == 0 ? bw4_of(mi(mvRow, mvCol).mi_size) : bh4_of(mi(mvRow, mvCol).mi_size);
        }
    }
    if (b.ref[1] > INTRA_FRAME) {
        MvList2 comb[2];
        for (int list = 0; list < 2; list++) {
            for (const Mv& m : idMvs[list]) comb[list].push_back(m);
            for (size_t i = 0; i < diffMvs[list].size() && comb[list].size() < 2; i++) comb[list].push_back(diffMvs[list][i]);
            while (comb[list].size() < 2) comb[list].push_back(s.global[list]);
        }
        if (s.num == 1) {
            if (comb[0][0] == s.stack[0][0] && comb[1][0] == s.stack[0][1]) {
                s.stack[s.num][0] = comb[0][1];
                s.stack[s.num][1] = comb[1][1];
            } else {
                s.stack[s.num][0] = comb[0][0];
                s.stack[s.num][1] = comb[1][0];
            }
            s.weight[s.num] = 2;
            s.num++;
        } else {
            for (int idx = 0; idx < 2; idx++) {
                s.stack[s.num][0] = comb[0][idx];
                s.stack[s.num][1] = comb[1][idx];
                s.weight[s.num] = 2;
                s.num++;
            }
        }
    } else {
        for (int idx = s.num; idx < 2; idx++) s.stack[idx][0] = s.global[0];
    }
}

void BlockParser::find_mv_stack(Blk& b, MvStack& s)
{
    const bool isCompound = b.ref[1] > INTRA_FRAME;
    s.num = 0;
    s.new_count = 0;
    setup_global_mv(b, s, 0);
    if (isCompound) setup_global_mv(b, s, 1);
    s.found = false;
    scan_row(b, s, -1);
    bool foundAbove = s.found;
    s.found = false;
    scan_col(b, s, -1);
    bool foundLeft = s.found;
    if (std::max(b.bw4, b.bh4) <= 16) {
        s.found = false;
        scan_point(b, s, -1, b.bw4);
        if (s.found) foundAbove = true;
    }
    const int closeMatches = foundAbove + foundLeft;
    const int numNearest = s.num, numNew = s.new_count;
    for (int i = 0; i < numNearest; i++) s.weight[i] += kRefCatLevel640;
    s.zero_ctx = 0;
    if (fh.use_ref_frame_mvs) temporal_scan(b, s);
    s.found = false;
    scan_point(b, s, -1, -1);
    if (s.found) {
        foundAbove = true;
        s.found = false;
    }
    scan_row(b, s, -3);
    if (s.found) {
        foundAbove = true;
        s.found = false;
    }
    scan_col(b, s, -3);
    if (s.found) {
        foundLeft = true;
        s.found = false;
    }
    if (b.bh4 > 1) {
        scan_row(b, s, -5);
        if (s.found) {
            foundAbove = true;
            s.found = false;
        }
    }
    if (b.bw4 > 1) {
        scan_col(b, s, -5);
        if (s.found) {
            foundLeft = true;
            s.found = false;
        }
    }
    const int totalMatches = foundAbove + foundLeft;
    auto sort = [&](int start, int end) {
        while (end > start) {
            int newEnd = start;
            for (int idx = start + 1; idx < end; idx++)
                if (s.weight[idx - 1] < s.weight[idx]) {
                    std::swap(s.weight[idx - 1], s.weight[idx]);
                    for (int l = 0; l < 1 + isCompound; l++) std::swap(s.stack[idx - 1][l], s.stack[idx][l]);
                    newEnd = idx;
                }
            end = newEnd;
        }
    };
    sort(0, numNearest);
    sort(numNearest, s.num);
    if (s.num < 2) extra_search(b, s);
    for (int idx = 0; idx < s.num; idx++) {
        uint8_t z = 0;
        if (idx + 1 < s.num) {
            const uint32_t w0 = s.weight[idx], w1 = s.weight[idx + 1];
            if (w0 >= (uint32_t)kRefCatLevel640) z = w1 < (uint32_t)kRefCatLevel640 ? 1 : 0;
            else z = 2;
        }
        s.drl_ctx[idx] = z;
    }
    if (closeMatches == 0) {
        s.new_ctx = std::min(totalMatches, 1);
        s.ref_ctx = totalMatches;
    } else if (closeMatches == 1) {
        s.new_ctx = 3 - std::min(numNew, 1);
        s.ref_ctx = 2 + totalMatches;
    } else {
        s.new_ctx = 5 - std::min(numNew, 1);
        s.ref_ctx = 5;
    }
    // clampMv (InterPredict.cpp:1469-1495)
    for (int list = 0; list < 1 + isCompound; list++)
        for (int idx = 0; idx < s.num; idx++) {
            Mv& m = s.stack[idx][list];
            const int toTop = -((b.r * 4) * 8), toBottom = ((fh.mi_rows - b.bh4 - b.r) * 4) * 8;
            const int toLeft = -((b.c * 4) * 8), toRight = ((fh.mi_cols - b.bw4 - b.c) * 4) * 8;
            const int br = kMvBorder + b.bh4 * 4 * 8, bc = kMvBorder + b.bw4 * 4 * 8;
            m.r = (int16_t)clip3(toTop - br, toBottom + br, m.r);
            m.c = (int16_t)clip3(toLeft - bc, toRight + bc, m.c);
        }
}

// ------------------------------------------------------------------------------------
// local warp (Block::LocalWarp, Block.cpp:957-1200)
// ------------------------------------------------------------------------------------
void BlockParser::add_sample(Blk& b, int deltaRow, int deltaCol)
{
    if (b.num_scanned >= 8) return;
    const int mvRow = b.r + deltaRow, mvCol = b.c + deltaCol;
    if (!inside(mvRow, mvCol)) return;
    const MiInfo& m = mi(mvRow, mvCol);
    if (m.ref[0] == NONE_FRAME || m.ref[0] != b.ref[0] || m.ref[1] != NONE_FRAME) return;
    const int candW4 = bw4_of(m.mi_size), candH4 = bh4_of(m.mi_size);
    const int candRow = mvRow & ~(candH4 - 1), candCol = mvCol & ~(candW4 - 1);
    const int midY = candRow * 4 + candH4 * 2 - 1, midX = candCol * 4 + candW4 * 2 - 1;
    const int threshold = clip3(16, 112, std::max(b.bw4 * 4, b.bh4 * 4));
    const MiInfo& cm = mi(candRow, candCol);
    const int mvDiffRow = abs(cm.mv[0].r - b.mv[0].r), mvDiffCol = abs(cm.mv[0].c - b.mv[0].c);
    const bool valid = mvDiffRow + mvDiffCol <= threshold;
    int cand[4] = {(int16_t)(midY * 8), (int16_t)(midX * 8), (int16_t)(midY * 8 + cm.mv[0].r), (int16_t)(midX * 8 + cm.mv[0].c)};
    b.num_scanned++;
    if (!valid && b.num_scanned > 1) return;
    memcpy(b.cand[b.num_samples], cand, sizeof(cand));
    if (valid) b.num_samples++;
}

void BlockParser::find_warp_samples(Blk& b)
{
    b.num_samples = b.num_scanned = 0;
    bool doTopLeft = true, doTopRight = true;
    if (b.avail_u) {
        const int srcW = bw4_of(mi(b.r - 1, b.c).mi_size);
        if (b.bw4 <= srcW) {
            const int colOffset = -(b.c & (srcW - 1));
            if (colOffset < 0) doTopLeft = false;
            if (colOffset + srcW > b.bw4) doTopRight = false;
            add_sample(b, -1, 0);
        } else {
            int step;
            for (int i = 0; i < std::min(b.bw4, fh.mi_cols - b.c); i += step) {
                step = std::min(b.bw4, bw4_of(mi(b.r - 1, b.c + i).mi_size));
                add_sample(b, -1, i);
            }
        }
    }
    if (b.avail_l) {
        const int srcH = bh4_of(mi(b.r, b.c - 1).mi_size);
        if (b.bh4 <= srcH) {
            const int rowOffset = -(b.r & (srcH - 1));
            if (rowOffset < 0) doTopLeft = false;
            add_sample(b, 0, -1);
        } else {
            int step;
            for (int i = 0; i < std::min(b.bh4, fh.mi_rows - b.r); i += step) {
                step = std::min(b.bh4, bh4_of(mi(b.r + i, b.c - 1).mi_size));
                add_sample(b, i, -1);
            }
        }
    }
    if (doTopLeft) add_sample(b, -1, -1);
    if (doTopRight && std::max(b.bw4, b.bh4) <= 16) add_sample(b, -1, b.bw4);
    if (b.num_samples == 0 && b.num_scanned > 0) b.num_samples = 1;
}

static void resolve_divisor(int64_t d, int& divShift, int& divFactor)
{
    const uint64_t ad = (uint64_t)(d < 0 ? -d : d);
    const int n = floor_log2(ad);
    const int64_t e = (int64_t)ad - ((int64_t)1 << n);
    const int64_t f = n > 8 ? round2_64(e, n - 8) : (e << (8 - n));
    divShift = n + 14;
    divFactor = d < 0 ? -(int)av1r_div_lut[f] : (int)av1r_div_lut[f];
}

void BlockParser::warp_estimation(Blk& b)  // warpEstimation + setupShear
{
    auto ls_product = [](int a, int c) { return ((a * c) >> 2) + (a + c); };
    int64_t A[2][2] = {{0, 0}, {0, 0}}, Bx[2] = {0, 0}, By[2] = {0, 0};
    const int midY = b.r * 4 + b.bh4 * 2 - 1, midX = b.c * 4 + b.bw4 * 2 - 1;
    const int suy = midY * 8, sux = midX * 8;
    const int duy = suy + b.mv[0].r, dux = sux + b.mv[0].c;
    for (int i = 0; i < b.num_samples; i++) {
        const int sy = b.cand[i][0] - suy, sx = b.cand[i][1] - sux;
        const int dy = b.cand[i][2] - duy, dx = b.cand[i][3] - dux;
        if (abs(sx - dx) < 256 && abs(sy - dy) < 256) {
            A[0][0] += ls_product(sx, sx) + 8;
            A[0][1] += ls_product(sx, sy) + 4;
            A[1][1] += ls_product(sy, sy) + 8;
            Bx[0] += ls_product(sx, dx) + 8;
            Bx[1] += ls_product(sy, dx) + 4;
            By[0] += ls_product(sx, dy) + 4;
            By[1] += ls_product(sy, dy) + 8;
        }
    }
    const int64_t det = A[0][0] * A[1][1] - A[0][1] * A[0][1];
    b.local_valid = det != 0;
    if (!b.local_valid) return;
    int divShift, divFactor;
    resolve_divisor(det, divShift, divFactor);
    divShift -= kWarpPrecBits;
    if (divShift < 0) {
        divFactor = divFactor * (1 << (-divShift));
        divShift = 0;
    }
    const int kClamp = 1 << 13;
    auto nondiag = [&](int64_t v) {
        return (int32_t)std::max<int64_t>(-kClamp + 1, std::min<int64_t>(kClamp - 1, round2signed_64(v * divFactor, divShift)));
    };
    auto diag = [&](int64_t v) {
        return (int32_t)std::max<int64_t>((1 << kWarpPrecBits) - kClamp + 1,
                                          std::min<int64_t>((1 << kWarpPrecBits) + kClamp - 1, round2signed_64(v * divFactor, divShift)));
    };
    int32_t* p = b.local_warp;
    p[2] = diag(A[1][1] * Bx[0] - A[0][1] * Bx[1]);
    p[3] = nondiag(-A[0][1] * Bx[0] + A[0][0] * Bx[1]);
    p[4] = nondiag(A[1][1] * By[0] - A[0][1] * By[1]);
    p[5] = diag(-A[0][1] * By[0] + A[0][0] * By[1]);
    const int vx = b.mv[0].c * (1 << (kWarpPrecBits - 3)) - (midX * (p[2] - (1 << kWarpPrecBits)) + midY * p[3]);
    const int vy = b.mv[0].r * (1 << (kWarpPrecBits - 3)) - (midX * p[4] + midY * (p[5] - (1 << kWarpPrecBits)));
    p[0] = clip3(-(1 << 23), (1 << 23) - 1, vx);
    p[1] = clip3(-(1 << 23), (1 << 23) - 1, vy);
    // setupShear (Block.cpp:1179-1200): the model must be representable as two shears
    const int alpha0 = clip3(-32768, 32767, p[2] - (1 << kWarpPrecBits));
    const int beta0 = clip3(-32768, 32767, p[3]);
    resolve_divisor(p[2], divShift, divFactor);
    const int64_t v = (int64_t)p[4] * (1 << kWarpPrecBits);
    const int gamma0 = (int)std::max<int64_t>(-32768, std::min<int64_t>(32767, round2signed_64(v * divFactor, divShift)));
    const int64_t w = (int64_t)p[3] * p[4];
    const int delta0 = (int)std::max<int64_t>(
        -32768, std::min<int64_t>(32767, p[5] - round2signed_64(w * divFactor, divShift) - (1 << kWarpPrecBits)));
    auto reduce = [](int x) { return (int)(round2signed_64(x, 6) * 64); };
    const int alpha = reduce(alpha0), beta = reduce(beta0), gamma = reduce(gamma0), delta = reduce(delta0);
    if (4 * abs(alpha) + 7 * abs(beta) >= (1 << kWarpPrecBits)) b.local_valid = false;
    if (4 * abs(gamma) + 4 * abs(delta) >= (1 << kWarpPrecBits)) b.local_valid = false;
}

// ------------------------------------------------------------------------------------
// palette (Block.cpp:1952-2271)
// ------------------------------------------------------------------------------------
int BlockParser::palette_cache(const Blk& b, int plane, uint8_t* cache)
{
    int aboveN = 0, leftN = 0;
    const uint8_t* above = nullptr;
    const uint8_t* left = nullptr;
    if ((b.r * 4) % 64) {
        const MiInfo& m = mi(b.r - 1, b.c);
        aboveN = m.pal_size[plane];
        if (aboveN) above = &T.pal_colors[m.pal_idx][plane * 8];
    }
    if (b.avail_l) {
        const MiInfo& m = mi(b.r, b.c - 1);
        leftN = m.pal_size[plane];
        if (leftN) left = &T.pal_colors[m.pal_idx][plane * 8];
    }
    int ai = 0, li = 0, n = 0;
    while (ai < aboveN && li < leftN) {
        const uint8_t aboveC = above[ai], leftC = left[li];
        if (leftC < aboveC) {
            if (n == 0 || leftC != cache[n - 1]) cache[n++] = leftC;
            li++;
        } else {
            if (n == 0 || aboveC != cache[n - 1]) cache[n++] = aboveC;
            ai++;
            if (leftC == aboveC) li++;
        }
    }
    for (; ai < aboveN; ai++)
        if (n == 0 || above[ai] != cache[n - 1]) cache[n++] = above[ai];
    for (; li < leftN; li++)
        if (n == 0 || left[li] != cache[n - 1]) cache[n++] = left[li];
    return n;
}

void BlockParser::palette_mode_info(Blk& b)
{
    const int bsizeCtx = av1r_miw_log2[b.bsize] + av1r_mih_log2[b.bsize] - 2;
    const int bitDepth = 8;
    auto clip1 = [](int v) { return (uint8_t)clip3(0, 255, v); };
    if (b.y_mode == DC_PRED) {
        int ctx = 0;
        if (b.avail_u && mi(b.r - 1, b.c).pal_size[0] > 0) ctx++;
        if (b.avail_l && mi(b.r, b.c - 1).pal_size[0] > 0) ctx++;
        if (S(cdf.mode.palette_y_mode[bsizeCtx + 2][ctx], 2)) {
            b.pal_y = S(cdf.mode.palette_y_size[bsizeCtx + 2], 7) + 2;
            uint8_t cache[16];
            const int cacheN = palette_cache(b, 0, cache);
            int idx = 0;
            for (int i = 0; i < cacheN && idx < b.pal_y; i++)
                if (L(1)) b.colors[0][idx++] = cache[i];
            if (idx < b.pal_y) b.colors[0][idx++] = (uint8_t)L(bitDepth);
            int paletteBits = 0;
            if (idx < b.pal_y) paletteBits = bitDepth - 3 + (int)L(2);
            while (idx < b.pal_y) {
                const int delta = (int)L(paletteBits) + 1;
                b.colors[0][idx] = clip1(b.colors[0][idx - 1] + delta);
                const int range = (1 << bitDepth) - b.colors[0][idx] - 1;
                paletteBits = std::min(paletteBits, ceil_log2((uint32_t)range));
                idx++;
            }
            std::sort(b.colors[0], b.colors[0] + b.pal_y);
        }
    }
    if (b.has_chroma && b.uv_mode == DC_PRED) {
        if (S(cdf.mode.palette_uv_mode[b.pal_y > 0 ? 1 : 0], 2)) {
            b.pal_uv = S(cdf.mode.palette_uv_size[bsizeCtx + 2], 7) + 2;
            uint8_t cache[16];
            const int cacheN = palette_cache(b, 1, cache);
            int idx = 0;
            for (int i = 0; i < cacheN && idx < b.pal_uv; i++)
                if (L(1)) b.colors[1][idx++] = cache[i];
            if (idx < b.pal_uv) b.colors[1][idx++] = (uint8_t)L(bitDepth);
            int paletteBits = 0;
            if (idx < b.pal_uv) paletteBits = bitDepth - 3 + (int)L(2);
            while (idx < b.pal_uv) {
                const int delta = (int)L(paletteBits);
                b.colors[1][idx] = clip1(b.colors[1][idx - 1] + delta);
                const int range = (1 << bitDepth) - b.colors[1][idx];
                paletteBits = std::min(paletteBits, ceil_log2((uint32_t)range));
                idx++;
            }
            std::sort(b.colors[1], b.colors[1] + b.pal_uv);
            if (L(1)) {  // delta_encode_palette_colors_v
                // the reference keeps maxVal in a uint8_t (Block.cpp:2130), so for 8-bit
                // video it is 0 and the wrap-around never applies: values clip to 0..255
                const int bits = bitDepth - 4 + (int)L(2);
                b.colors[2][0] = (uint8_t)L(bitDepth);
                for (idx = 1; idx < b.pal_uv; idx++) {
                    int delta = (int)L(bits);
                    if (delta && L(1)) delta = -delta;
                    b.colors[2][idx] = clip1(b.colors[2][idx - 1] + delta);
                }
            } else {
                for (idx = 0; idx < b.pal_uv; idx++) b.colors[2][idx] = (uint8_t)L(bitDepth);
            }
        }
    }
}

static void color_context(const uint8_t* map, int stride, int r, int c, int n, uint8_t* order, int& hash)
{
    int scores[8];
    for (int i = 0; i < 8; i++) {
        scores[i] = 0;
        order[i] = (uint8_t)i;
    }
    if (c > 0) scores[map[r * stride + c - 1]] += 2;
    if (r > 0 && c > 0) scores[map[(r - 1) * stride + c - 1]] += 1;
    if (r > 0) scores[map[(r - 1) * stride + c]] += 2;
    for (int i = 0; i < 3; i++) {
        int maxScore = scores[i], maxIdx = i;
        for (int j = i + 1; j < n; j++)
            if (scores[j] > maxScore) {
                maxScore = scores[j];
                maxIdx = j;
            }
        if (maxIdx != i) {
            maxScore = scores[maxIdx];
            const uint8_t maxOrder = order[maxIdx];
            for (int k = maxIdx; k > i; k--) {
                scores[k] = scores[k - 1];
                order[k] = order[k - 1];
            }
            scores[i] = maxScore;
            order[i] = maxOrder;
        }
    }
    static const int mult[3] = {1, 2, 2};
    hash = 0;
    for (int i = 0; i < 3; i++) hash += scores[i] * mult[i];
}

void BlockParser::palette_tokens(Blk& b)
{
    const int bw = b.bw4 * 4, bh = b.bh4 * 4;
    int onW = std::min(bw, (fh.mi_cols - b.c) * 4), onH = std::min(bh, (fh.mi_rows - b.r) * 4);
    auto tokens = [&](std::vector<uint8_t>& map, int w, int h, int ow, int oh, int n, bool uv) {
        map.assign((size_t)w * h, 0);
        map[0] = (uint8_t)sd.ns((uint32_t)n);
        uint8_t order[8];
        int hash;
        for (int i = 1; i < oh + ow - 1; i++)
            for (int j = std::min(i, ow - 1); j >= std::max(0, i - oh + 1); j--) {
                color_context(map.data(), w, i - j, j, n, order, hash);
                const int ctx = kPaletteColorContext[hash];
                uint16_t* c = uv ? cdf.mode.palette_uv_color_index[n - 2][ctx] : cdf.mode.palette_y_color_index[n - 2][ctx];
                map[(size_t)(i - j) * w + j] = order[S(c, n)];
            }
        for (int i = 0; i < oh; i++)
            for (int j = ow; j < w; j++) map[(size_t)i * w + j] = map[(size_t)i * w + ow - 1];
        for (int i = oh; i < h; i++)
            for (int j = 0; j < w; j++) map[(size_t)i * w + j] = map[(size_t)(oh - 1) * w + j];
    };
    if (b.pal_y) {
        b.map_wy = bw;
        b.map_hy = bh;
        tokens(b.map_y, bw, bh, onW, onH, b.pal_y, false);
    }
    if (b.pal_uv) {
        int w = bw >> 1, h = bh >> 1;
        onW >>= 1;
        onH >>= 1;
        if (w < 4) {
            w += 2;
            onW += 2;
        }
        if (h < 4) {
            h += 2;
            onH += 2;
        }
        b.map_wuv = w;
        b.map_huv = h;
        tokens(b.map_uv, w, h, onW, onH, b.pal_uv, true);
    }
}

// ------------------------------------------------------------------------------------
// transform size (Block.cpp:1468-1598)
// ------------------------------------------------------------------------------------
int BlockParser::above_tx_width(const Blk& b, int row, int col)
{
    if (row == b.r) {
        if (!b.avail_u) return 64;
        const MiInfo& m = mi(row - 1, col);
        if (m.skip && m.is_inter) return bw4_of(m.mi_size) * 4;
    }
    return av1r_tx_w[mi(row - 1, col).inter_tx];
}

int BlockParser::left_tx_height(const Blk& b, int row, int col)
{
    if (col == b.c) {
        if (!b.avail_l) return 64;
        const MiInfo& m = mi(row, col - 1);
        if (m.skip && m.is_inter) return bh4_of(m.mi_size) * 4;
    }
    return av1r_tx_h[mi(row, col - 1).inter_tx];
}

void BlockParser::read_tx_size(Blk& b, bool allowSelect)
{
    if (b.lossless) {
        b.tx_size = TX_4X4;
        return;
    }
    const int maxRect = kMaxTxSizeRect[b.bsize];
    const int maxDepth = kMaxTxDepth[b.bsize];
    b.tx_size = maxRect;
    if (b.bsize > BLOCK_4X4 && allowSelect && fh.tx_mode == TX_MODE_SELECT) {
        int aboveW = 0, leftH = 0;
        if (b.avail_u) {
            const MiInfo& m = mi(b.r - 1, b.c);
            aboveW = m.is_inter ? bw4_of(m.mi_size) * 4 : above_tx_width(b, b.r, b.c);
        }
        if (b.avail_l) {
            const MiInfo& m = mi(b.r, b.c - 1);
            leftH = m.is_inter ? bh4_of(m.mi_size) * 4 : left_tx_height(b, b.r, b.c);
        }
        const int ctx = (aboveW >= av1r_tx_w[maxRect]) + (leftH >= av1r_tx_h[maxRect]);
        static const int depthToCat[5] = {0, 0, 1, 2, 3};
        const int cat = depthToCat[maxDepth];
        const int depth = S(cdf.mode.tx_size[cat][ctx], cat == 0 ? 2 : 3);
        for (int i = 0; i < depth; i++) b.tx_size = kSplitTxSize[b.tx_size];
    }
}

void BlockParser::read_var_tx_size(Blk& b, int row, int col, int txSz, int depth)
{
    if (row >= fh.mi_rows || col >= fh.mi_cols) return;
    bool split = false;
    if (!(txSz == TX_4X4 || depth == 2)) {
        const int above = above_tx_width(b, row, col) < av1r_tx_w[txSz];
        const int left = left_tx_height(b, row, col) < av1r_tx_h[txSz];
        const int size = std::min(64, std::max(bw4_of(b.bsize), bh4_of(b.bsize)) * 4);
        const int maxTxSz = find_tx_size(size, size);
        const int ctx = (kTxSizeSqrUp[txSz] != maxTxSz) * 3 + (4 - maxTxSz) * 6 + above + left;
        split = S(cdf.mode.txfm_partition[ctx], 2) != 0;
    }
    const int w4 = av1r_tx_w[txSz] / 4, h4 = av1r_tx_h[txSz] / 4;
    if (split) {
        const int sub = kSplitTxSize[txSz];
        const int stepW = av1r_tx_w[sub] / 4, stepH = av1r_tx_h[sub] / 4;
        for (int i = 0; i < h4; i += stepH)
            for (int j = 0; j < w4; j += stepW) read_var_tx_size(b, row + i, col + j, sub, depth + 1);
    } else {
        for (int i = 0; i < h4; i++)
            for (int j = 0; j < w4; j++) mi(row + i, col + j).inter_tx = (uint8_t)txSz;
        b.tx_size = txSz;
    }
}

void BlockParser::read_block_tx_size(Blk& b)
{
    if (fh.tx_mode == TX_MODE_SELECT && b.bsize > BLOCK_4X4 && b.is_inter && !b.skip && !fh.coded_lossless) {
        const int maxTx = kMaxTxSizeRect[b.bsize];
        const int txW4 = av1r_tx_w[maxTx] / 4, txH4 = av1r_tx_h[maxTx] / 4;
        for (int row = b.r; row < b.r + b.bh4; row += txH4)
            for (int col = b.c; col < b.c + b.bw4; col += txW4) read_var_tx_size(b, row, col, maxTx, 0);
    } else {
        read_tx_size(b, !b.skip || !b.is_inter);
        for (int row = b.r; row < b.r + b.bh4; row++)
            for (int col = b.c; col < b.c + b.bw4; col++) mi(row, col).inter_tx = (uint8_t)b.tx_size;
    }
}

void BlockParser::reset_block_context(const Blk& b)
{
    for (int plane = 0; plane < 1 + 2 * b.has_chroma; plane++) {
        const int sub = plane ? 1 : 0;
        std::fill_n(&T.above_level[plane][b.c >> sub], b.bw4 >> sub, 0);
        std::fill_n(&T.above_dc[plane][b.c >> sub], b.bw4 >> sub, 0);
        std::fill_n(&T.left_level[plane][b.r >> sub], b.bh4 >> sub, 0);
        std::fill_n(&T.left_dc[plane][b.r >> sub], b.bh4 >> sub, 0);
    }
}

// ------------------------------------------------------------------------------------
// residual (Block.cpp:176-301) and transform blocks (TransformBlock.cpp)
// ------------------------------------------------------------------------------------
int BlockParser::uv_tx_size(const Blk& b) const  // Block::get_tx_size for plane > 0
{
    const int uvTx = kMaxTxSizeRect[av1r_ss420[b.bsize]];
    if (av1r_tx_w[uvTx] == 64 || av1r_tx_h[uvTx] == 64) {
        if (av1r_tx_w[uvTx] == 16) return TX_16X32;
        if (av1r_tx_h[uvTx] == 16) return TX_32X16;
        return TX_32X32;
    }
    return uvTx;
}

void BlockParser::residual(Blk& b)
{
    const int widthChunks = std::max(1, (b.bw4 * 4) >> 6), heightChunks = std::max(1, (b.bh4 * 4) >> 6);
    const int sizeChunk = (widthChunks > 1 || heightChunks > 1) ? BLOCK_64X64 : b.bsize;
    for (int cy = 0; cy < heightChunks; cy++)
        for (int cx = 0; cx < widthChunks; cx++) {
            const int rowChunk = b.r + (cy << 4), colChunk = b.c + (cx << 4);
            for (int plane = 0; plane < 1 + b.has_chroma * 2; plane++) {
                const int txSz = b.lossless ? TX_4X4 : plane ? uv_tx_size(b) : b.tx_size;
                const int stepX = av1r_tx_w[txSz] >> 2, stepY = av1r_tx_h[txSz] >> 2;
                const int planeSz = plane ? av1r_ss420[sizeChunk] : sizeChunk;
                const int n4w = bw4_of(planeSz), n4h = bh4_of(planeSz);
                const int sub = plane ? 1 : 0;
                if (b.is_inter && !b.lossless && !plane) {
                    transform_tree(b, (colChunk >> sub) * 4, (rowChunk >> sub) * 4, n4w * 4, n4h * 4);
                } else {
                    const int baseX = (b.c >> sub) * 4, baseY = (b.r >> sub) * 4;
                    for (int y = 0; y < n4h; y += stepY)
                        for (int x = 0; x < n4w; x += stepX)
                            transform_block(b, plane, baseX, baseY, txSz, x + ((cx << 4) >> sub), y + ((cy << 4) >> sub));
                }
                if (!T.err.empty()) return;
            }
        }
}

void BlockParser::transform_tree(Blk& b, int startX, int startY, int w, int h)
{
    if (startX >= fh.mi_cols * 4 || startY >= fh.mi_rows * 4) return;
    const int lumaTx = mi(startY >> 2, startX >> 2).inter_tx;
    if (w <= av1r_tx_w[lumaTx] && h <= av1r_tx_h[lumaTx]) {
        transform_block(b, 0, startX, startY, find_tx_size(w, h), 0, 0);
    } else if (w > h) {
        transform_tree(b, startX, startY, w / 2, h);
        transform_tree(b, startX + w / 2, startY, w / 2, h);
    } else if (w < h) {
        transform_tree(b, startX, startY, w, h / 2);
        transform_tree(b, startX, startY + h / 2, w, h / 2);
    } else {
        transform_tree(b, startX, startY, w / 2, h / 2);
        transform_tree(b, startX + w / 2, startY, w / 2, h / 2);
        transform_tree(b, startX, startY + h / 2, w / 2, h / 2);
        transform_tree(b, startX + w / 2, startY + h / 2, w / 2, h / 2);
    }
}

// transform_block: the specification's bound (maxX = (MiCols * MI_SIZE) >> subX); the
// reference tests the luma bound for every plane (Block.cpp:188-191), which differs only
// for chroma blocks wholly outside the frame -- none of the conformance streams has one
void BlockParser::transform_block(Blk& b, int plane, int baseX, int baseY, int txSz, int x, int y)
{
    const int startX = baseX + 4 * x, startY = baseY + 4 * y;
    const int sub = plane ? 1 : 0;
    if (startX >= ((fh.mi_cols * 4) >> sub) || startY >= ((fh.mi_rows * 4) >> sub)) return;
    Tb t;
    t.plane = plane;
    t.x = startX;
    t.y = startY;
    t.base_x = baseX;
    t.base_y = baseY;
    t.tx = txSz;
    t.eob = 0;
    t.type = 0;
    t.coef_off = (uint32_t)T.coefs.size();
    t.coef_cnt = 0;
    const int x4 = startX >> 2, y4 = startY >> 2, w4 = av1r_tx_w[txSz] >> 2, h4 = av1r_tx_h[txSz] >> 2;
    if (b.skip) {
        std::fill_n(&T.above_level[plane][x4], w4, 0);
        std::fill_n(&T.above_dc[plane][x4], w4, 0);
        std::fill_n(&T.left_level[plane][y4], h4, 0);
        std::fill_n(&T.left_dc[plane][y4], h4, 0);
    } else {
        t.eob = coeffs(b, t);
    }
    tbs.push_back(t);
}

int BlockParser::tx_set(const Blk& b, int txSz) const  // TransformBlock::get_tx_set
{
    const int sqrUp = kTxSizeSqrUp[txSz], sqr = kTxSizeSqr[txSz];
    if (sqrUp > TX_32X32) return TX_SET_DCTONLY;
    if (b.is_inter) {
        if (fh.reduced_tx_set || sqrUp == TX_32X32) return TX_SET_3;
        if (sqr == 2) return TX_SET_2;
        return TX_SET_1;
    }
    if (sqrUp == TX_32X32) return TX_SET_DCTONLY;
    if (fh.reduced_tx_set) return TX_SET_2;
    if (sqr == 2) return TX_SET_2;
    return TX_SET_1;
}

int BlockParser::compute_tx_type(const Blk& b, int plane, int txSz, int x4, int y4) const
{
    if (b.lossless || kTxSizeSqrUp[txSz] > TX_32X32) return DCT_DCT;
    const int set = tx_set(b, txSz);
    if (plane == 0) return P.mi[(size_t)y4 * P.mi_stride + x4].tx_type;
    auto inSet = [&](int type) { return b.is_inter ? kTxInSetInter[set][type] : kTxInSetIntra[set][type]; };
    if (b.is_inter) {
        const int i = std::max(b.c, x4 << 1), j = std::max(b.r, y4 << 1);
        const int type = P.mi[(size_t)j * P.mi_stride + i].tx_type;
        return inSet(type) ? type : DCT_DCT;
    }
    const int type = kModeToTxfm[b.uv_mode];
    return inSet(type) ? type : DCT_DCT;
}

int BlockParser::all_zero_ctx(const Blk& b, int plane, int txSz, int x4, int y4, int w, int h) const
{
    int maxX4 = fh.mi_cols, maxY4 = fh.mi_rows;
    if (plane) {
        maxX4 >>= 1;
        maxY4 >>= 1;
    }
    const int bsz = plane ? av1r_ss420[b.bsize] : b.bsize;
    const int bw = bw4_of(bsz) * 4, bh = bh4_of(bsz) * 4;
    const int w4 = w >> 2, h4 = h >> 2;
    (void)txSz;
    if (plane == 0) {
        int top = 0, left = 0;
        for (int k = 0; k < w4; k++)
            if (x4 + k < maxX4) top = std::max(top, (int)T.above_level[plane][x4 + k]);
        for (int k = 0; k < h4; k++)
            if (y4 + k < maxY4) left = std::max(left, (int)T.left_level[plane][y4 + k]);
        top = std::min(top, 255);
        left = std::min(left, 255);
        if (bw == w && bh == h) return 0;
        if (top == 0 && left == 0) return 1;
        if (top == 0 || left == 0) return 2 + (std::max(top, left) > 3);
        if (std::max(top, left) <= 3) return 4;
        if (std::min(top, left) <= 3) return 5;
        return 6;
    }
    int above = 0, left = 0;
    for (int i = 0; i < w4; i++)
        if (x4 + i < maxX4) above |= T.above_level[plane][x4 + i] | T.above_dc[plane][x4 + i];
    for (int i = 0; i < h4; i++)
        if (y4 + i < maxY4) left |= T.left_level[plane][y4 + i] | T.left_dc[plane][y4 + i];
    int ctx = (above != 0) + (left != 0) + 7;
    if (bw * bh > w * h) ctx += 3;
    return ctx;
}

// TransformBlock::coeffs (TransformBlock.cpp:1637-1704) + transform_type (1271-1327)
int BlockParser::coeffs(Blk& b, Tb& t)
{
    const int txSz = t.tx, plane = t.plane, ptype = plane > 0;
    const int x4 = t.x >> 2, y4 = t.y >> 2;
    const int w = av1r_tx_w[txSz], h = av1r_tx_h[txSz], w4 = w >> 2, h4 = h >> 2;
    const int sqr = kTxSizeSqr[txSz], sqrUp = kTxSizeSqrUp[txSz];
    const int txSzCtx = (sqr + sqrUp + 1) >> 1;
    const int tw = std::min(w, 32);
    const int segEob = (txSz == TX_16X64 || txSz == TX_64X16) ? 512 : std::min(1024, w * h);
    // quant[] is all zero between transform blocks: each block clears what it set
    if (quant.size() != 1024) quant.assign(1024, 0);
    (void)segEob;
    int eob = 0, culLevel = 0, dcCategory = 0;
    auto set_luma_type = [&](int type) {
        for (int i = 0; i < w4; i++)
            for (int j = 0; j < h4; j++) P.mi[(size_t)(y4 + j) * P.mi_stride + x4 + i].tx_type = (uint8_t)type;
    };
    PROF_T(c0);
    const int azCtx = all_zero_ctx(b, plane, txSz, x4, y4, w, h);
#ifdef AV1P_TRACE
    {
        static FILE* tf = fopen("/tmp/av1p_az.txt", "w");
        fprintf(tf, "p%d x4 %d y4 %d tx %d ctx %d\n", plane, x4, y4, txSz, azCtx);
    }
#endif
    const bool allZero = SN<2>(cdf.coef.txb_skip[txSzCtx][azCtx]) != 0;
    if (allZero) {
        if (plane == 0) set_luma_type(DCT_DCT);
    } else {
        if (plane == 0) {
            const int set = tx_set(b, txSz);
            int type = DCT_DCT;
            const int qidx = fh.base_q_idx;  // get_q_idx(): segmentation is rejected
            if (set > 0 && qidx > 0) {
                if (b.is_inter) {
                    const int nsym = set == TX_SET_1 ? 16 : set == TX_SET_2 ? 12 : 2;
                    const int s = S(cdf.mode.inter_ext_tx[set][sqr], nsym);
                    type = set == TX_SET_1 ? kInterInvSet1[s] : set == TX_SET_2 ? kInterInvSet2[s] : (s ? DCT_DCT : IDTX);
                } else {
                    const int dir = b.use_filter_intra ? kFilterIntraModeToIntraDir[b.filter_intra_mode] : b.y_mode;
                    const int nsym = set == TX_SET_1 ? 7 : 5;
                    const int s = S(cdf.mode.intra_ext_tx[set][sqr][dir], nsym);
                    type = set == TX_SET_1 ? kIntraInvSet1[s] : kIntraInvSet2[s];
                }
            }
            set_luma_type(type);
        }
        PROF_T(c1);
        PROF_ADD(4, c0, c1);
        t.type = compute_tx_type(b, plane, txSz, x4, y4);
        const int cls = tx_class(t.type);
        // eob (TransformBlock::getEob, 1440-1460)
        const int eobMultisize = std::min(av1r_tx_w_log2[txSz], (uint8_t)5) + std::min(av1r_tx_h_log2[txSz], (uint8_t)5) - 4;
        const int eobCtx = cls == TX_CLASS_2D ? 0 : 1;
        uint16_t* ec;
        switch (eobMultisize) {
        case 0: ec = cdf.coef.eob_flag_cdf16[ptype][eobCtx]; break;
        case 1: ec = cdf.coef.eob_flag_cdf32[ptype][eobCtx]; break;
        case 2: ec = cdf.coef.eob_flag_cdf64[ptype][eobCtx]; break;
        case 3: ec = cdf.coef.eob_flag_cdf128[ptype][eobCtx]; break;
        case 4: ec = cdf.coef.eob_flag_cdf256[ptype][eobCtx]; break;
        case 5: ec = cdf.coef.eob_flag_cdf512[ptype][eobCtx]; break;
        default: ec = cdf.coef.eob_flag_cdf1024[ptype][eobCtx]; break;
        }
        const int eobPt = S(ec, eobMultisize + 5) + 1;
        eob = eobPt < 2 ? eobPt : (1 << (eobPt - 2)) + 1;
        int eobShift = std::max(-1, eobPt - 3);
        if (eobShift >= 0) {
            if (SN<2>(cdf.coef.eob_extra[txSzCtx][ptype][eobPt - 3])) eob += 1 << eobShift;
            for (int i = 1; i < std::max(0, eobPt - 2); i++) {
                eobShift = std::max(0, eobPt - 2) - 1 - i;
                if (L(1)) eob += 1 << eobShift;
            }
        }
        PROF_T(c2);
        PROF_ADD(5, c1, c2);
        // levels, in reverse scan order
        const int adj = kAdjustedTxSize[txSz];
        const int bwl = av1r_tx_w_log2[adj];
        const int width = 1 << bwl, height = av1r_tx_h[adj];
        // levels so far, padded by 4 zero rows / columns below and right (every context offset
        // is non-negative): the neighbour sums need no bounds checks.  Each entry holds
        // level << 8 | min(level, 3), and the range context's 3 neighbours are the first 3 of
        // the base context's 5 (both offset lists of the spec, for every class), so one pass of
        // 16-bit sums gives both: the 5-sum's low byte (<= 15) the base magnitude, the 3-sum's
        // high byte the range magnitude
        const int ps = width + 4;
        int off[5];  // kSigRefDiffOffset in lvl[] units (per transform block, not per level)
        for (int k = 0; k < 5; k++) off[k] = kSigRefDiffOffset[cls][k][0] * ps + kSigRefDiffOffset[cls][k][1];
        const ScanEntry* se = kScanTables.t[txSz][cls].data();
        uint16_t* const cb = cdf.coef.coeff_base[txSzCtx][ptype][0];
        uint16_t* const cbr = cdf.coef.coeff_br[std::min(txSzCtx, 3)][ptype][0];
        constexpr int kCbStride = sizeof(cdf.coef.coeff_base[0][0][0]) / sizeof(uint16_t);
        constexpr int kBrStride = sizeof(cdf.coef.coeff_br[0][0][0]) / sizeof(uint16_t);
        int nnz = 0;
        for (int c = eob - 1; c >= 0; c--) {
            const ScanEntry e = se[c];
            uint16_t* lp = &lvl[e.pad];
            const uint32_t s3 = (uint32_t)lp[off[0]] + lp[off[1]] + lp[off[2]];
            int level;
            if (c == eob - 1) {
                int ctx;
                if (c == 0) ctx = kSigCoefContexts - 4;
                else if (c <= (height << bwl) / 8) ctx = kSigCoefContexts - 3;
                else if (c <= (height << bwl) / 4) ctx = kSigCoefContexts - 2;
                else ctx = kSigCoefContexts - 1;
                ctx = ctx - kSigCoefContexts + kSigCoefContextsEob;
                level = SN<3>(cdf.coef.coeff_base_eob[txSzCtx][ptype][ctx]) + 1;
            } else {
                const uint32_t mag = (s3 + lp[off[3]] + lp[off[4]]) & 0xff;
                const int ctx = (e.base & 0x80) ? 0 : std::min((int)(mag + 1) >> 1, 4) + e.base;
                level = SN<4>(cb + ctx * kCbStride);
            }
            if (level > kNumBaseLevels) {
                const int ctx = std::min((int)((s3 >> 8) + 1) >> 1, 6) + e.br;
                uint16_t* const bc = cbr + ctx * kBrStride;
                for (int idx = 0; idx < kCoeffBaseRange / (kBrCdfSize - 1); idx++) {
                    const int br = SN<4>(bc);
                    level += br;
                    if (br < kBrCdfSize - 1) break;
                }
            }
            quant[e.pos] = level;
            *lp = (uint16_t)(level << 8 | std::min(level, 3));
            nzc[nnz] = (uint16_t)c;
            nnz += level != 0;
        }
        for (int q = 0; q < nnz; q++) lvl[se[nzc[q]].pad] = 0;  // back to all zero for the next transform block (zero levels stored 0)
        (void)height;
        PROF_T(c3);
        PROF_ADD(6, c2, c3);
        // signs and Golomb remainders of the non-zero levels, in scan order (nzc from its end);
        // the non-zero positions also into a bitmap of rows (the packing below walks only them)
        const int twl = av1r_tx_w_log2[txSz] < 5 ? av1r_tx_w_log2[txSz] : 5;  // log2(tw)
        uint32_t nzRow[32] = {}, rowMask = 0;
        for (int q = nnz - 1; q >= 0; q--) {
            const int c = nzc[q];
            const int pos = se[c].pos;
            bool sign = false;
            {
                if (c == 0) {
                    int maxX4 = fh.mi_cols, maxY4 = fh.mi_rows;
                    if (plane) {
                        maxX4 >>= 1;
                        maxY4 >>= 1;
                    }
                    int dcSign = 0;
                    for (int k = 0; k < w4; k++)
                        if (x4 + k < maxX4) {
                            const int s = T.above_dc[plane][x4 + k];
                            dcSign += s == 1 ? -1 : s == 2 ? 1 : 0;
                        }
                    for (int k = 0; k < h4; k++)
                        if (y4 + k < maxY4) {
                            const int s = T.left_dc[plane][y4 + k];
                            dcSign += s == 1 ? -1 : s == 2 ? 1 : 0;
                        }
                    const int ctx = dcSign < 0 ? 1 : dcSign > 0 ? 2 : 0;
                    sign = SN<2>(cdf.coef.dc_sign[ptype][ctx]) != 0;
                } else {
                    sign = L(1) != 0;
                }
            }
            if (quant[pos] > kNumBaseLevels + kCoeffBaseRange) {
                int length = 0;
                uint32_t bit;
                do {
                    length++;
#ifdef AV1P_WRITER
                    if (sd.hook) sd.hook->golomb_prefix(length);
#endif
                    bit = L(1);
                    if (length > 32) {
                        T.fail(AV1R_E_INVALID, "invalid Golomb code");
                        return 0;
                    }
                } while (!bit);
                uint32_t x = 1;
                for (int i = length - 2; i >= 0; i--) x = (x << 1) | L(1);
                // int16 twice, as the reference's getLevel (TransformBlock.cpp:1620-1635)
                quant[pos] = (int16_t)((int16_t)x + kCoeffBaseRange + kNumBaseLevels);
            }
            if (pos == 0 && quant[pos] > 0) dcCategory = sign ? 1 : 2;
            if (quant[pos]) {
                nzRow[pos >> twl] |= 1u << (pos & (tw - 1));
                rowMask |= 1u << (pos >> twl);
            }
            culLevel += quant[pos];
            if (sign) quant[pos] = -quant[pos];
        }
#ifdef AV1P_TRACE
        {
            static FILE* tf = fopen("/tmp/av1p_cul.txt", "w");
            fprintf(tf, "p%d x4 %d y4 %d eob %d cul %d\n", plane, x4, y4, eob, culLevel);
        }
#endif
        culLevel = std::min(63, culLevel);
        PROF_T(c4);
        PROF_ADD(7, c3, c4);
        // packed non-zero coefficients (refdump.cpp dumpBlock), Quant[] layout i * tw + j, in
        // raster order (the rows' bitmaps, lowest bit first), cleared again
        std::vector<uint32_t>& out = T.coefs;
        out.resize(t.coef_off + nnz);
        uint32_t* o = out.data() + t.coef_off;
        for (uint32_t rm = rowMask; rm; rm &= rm - 1) {  // the rows holding a non-zero level, in order
            const int i = __builtin_ctz(rm);
            int* row = &quant[i * tw];
            for (uint32_t m = nzRow[i]; m; m &= m - 1) {
                const int j = __builtin_ctz(m);
                const int v = row[j];
                row[j] = 0;
                if (v >= (1 << 21) || v < -(1 << 21)) {
                    T.fail(AV1R_E_UNSUPPORTED, "coefficient out of packable range");
                    return 0;
                }
                *o++ = ((uint32_t)v << 10) | (uint32_t)(i * tw + j);
            }
        }
        out.resize((size_t)(o - out.data()));
        t.coef_cnt = (uint32_t)out.size() - t.coef_off;
#ifdef AV1P_PROF
        {
            PROF_T(c6);
            PROF_ADD(8, c4, c6);
        }
#endif
        if (!t.coef_cnt) {
            T.fail(AV1R_E_INVALID, "transform block with eob %d and no non-zero coefficient", eob);
            return 0;
        }
    }
#ifdef AV1P_PROF
    {
        PROF_T(c5);
        PROF_ADD(9, c0, c5);
    }
#endif
    std::fill_n(&T.above_level[plane][x4], w4, (int16_t)culLevel);
    std::fill_n(&T.above_dc[plane][x4], w4, (uint8_t)dcCategory);
    std::fill_n(&T.left_level[plane][y4], h4, (int16_t)culLevel);
    std::fill_n(&T.left_dc[plane][y4], h4, (uint8_t)dcCategory);
    return eob;
}

// ------------------------------------------------------------------------------------
// batch records (refdump.cpp dumpBlock) + the decode-time state they read
// ------------------------------------------------------------------------------------
void BlockParser::emit(Blk& b)
{
    TileCtx& F = T;  // (records tile-relative until merge_tile)
    const uint32_t blockIdx = (uint32_t)F.blocks.size();
    F.blocks.emplace_back();  // (value-initialised, i.e. zeroed, and written in place)
    av1r_block& rec = F.blocks.back();
    rec.mi_row = (uint16_t)b.r;
    rec.mi_col = (uint16_t)b.c;
    rec.mi_size = (uint8_t)b.bsize;
    rec.qindex = (uint8_t)(fh.delta_q_present ? b.qindex : fh.base_q_idx);
    rec.y_mode = (uint8_t)b.y_mode;
    // only the values reconstruction reads for this kind of block (the rest is 0)
    rec.uv_mode = (uint8_t)((b.has_chroma && !b.is_inter) ? b.uv_mode : 0);
    rec.angle_delta_y = (int8_t)b.angle_y;
    rec.angle_delta_uv = (int8_t)b.angle_uv;
    rec.filter_intra_mode = (uint8_t)((!b.is_inter && b.use_filter_intra) ? b.filter_intra_mode : 0);
    if (!b.is_inter && b.has_chroma && b.uv_mode == UV_CFL_PRED) {
        rec.cfl_alpha_u = (int8_t)b.cfl_u;
        rec.cfl_alpha_v = (int8_t)b.cfl_v;
    }
    rec.palette_size_y = (uint8_t)b.pal_y;
    rec.palette_size_uv = (uint8_t)b.pal_uv;
    {  // the block's mode info as stored over its 4x4 units (decode_block above)
        const MiInfo& m = mi(b.r, b.c);
        for (int l = 0; l < 2; l++) {
            rec.mv[l][0] = m.mv[l].r;
            rec.mv[l][1] = m.mv[l].c;
            rec.ref_frame[l] = m.ref[l];
        }
        rec.filt = (uint8_t)((m.interp[0] & 15) | (m.interp[1] << 4));
        for (int i = 0; i < 4; i++) rec.delta_lf[i] = (int8_t)T.delta_lf[i];  // (the block's, as stored over its units)
    }
    uint32_t f = 0;
    const bool ii = b.is_inter && b.interintra && !b.use_intrabc;
    if (b.is_inter) {
        f |= AV1R_BLK_INTER;
        rec.motion_mode = (uint8_t)b.motion_mode;
        rec.compound_type = (uint8_t)b.compound_type;
        rec.interintra_mode = (uint8_t)(ii ? b.interintra_mode : 0);
        if (b.compound_type == COMPOUND_WEDGE) {
            rec.wedge_index = (uint8_t)b.wedge_index;
            rec.wedge_sign = (uint8_t)b.wedge_sign;
        }
        if (b.compound_type == COMPOUND_DIFFWTD) rec.mask_type = b.mask_type;
        if (ii) f |= AV1R_BLK_INTERINTRA;
        if (ii && b.wedge_interintra) f |= AV1R_BLK_WEDGE_II;
    }
    if (b.use_intrabc) f |= AV1R_BLK_INTRABC;
    if (b.lossless) f |= AV1R_BLK_LOSSLESS;
    if (b.has_chroma) f |= AV1R_BLK_HAS_CHROMA;
    if (!b.is_inter && b.use_filter_intra) f |= AV1R_BLK_FILTER_INTRA;
    if (b.avail_l) f |= AV1R_BLK_AVAIL_L;
    if (b.avail_u) f |= AV1R_BLK_AVAIL_U;
    if (b.avail_l_uv) f |= AV1R_BLK_AVAIL_L_UV;
    if (b.avail_u_uv) f |= AV1R_BLK_AVAIL_U_UV;
    if (b.skip) f |= AV1R_BLK_SKIP;
    if (!b.is_inter) {
        // IntraPredict getAboveSmooth / getLeftSmooth (IntraPredict.cpp:211-260)
        auto smooth = [&](int plane, int r, int c) {
            const MiInfo& m = mi(r, c);
            int mode;
            if (!plane) {
                mode = m.y_mode;
            } else {
                if (m.ref[0] > INTRA_FRAME) return false;
                mode = m.uv_mode;
            }
            return mode == SMOOTH_PRED || mode == SMOOTH_V_PRED || mode == SMOOTH_H_PRED;
        };
        for (int plane = 0; plane < 2; plane++) {
            if (plane ? b.avail_u_uv : b.avail_u) {
                int r = b.r - 1, c = b.c;
                if (plane) {
                    if (!(b.c & 1)) c++;
                    if (b.r & 1) r--;
                }
                if (smooth(plane, r, c)) f |= plane ? AV1R_BLK_SMOOTH_A_UV : AV1R_BLK_SMOOTH_A_Y;
            }
            if (plane ? b.avail_l_uv : b.avail_l) {
                int r = b.r, c = b.c - 1;
                if (plane) {
                    if (b.c & 1) c--;
                    if (!(b.r & 1)) r++;
                }
                if (smooth(plane, r, c)) f |= plane ? AV1R_BLK_SMOOTH_L_UV : AV1R_BLK_SMOOTH_L_Y;
            }
        }
    }
    const int sbMask = seq.use_128x128 ? 31 : 15;
    if (b.is_inter && b.ref[1] == INTRA_FRAME) {  // block-level interintra edges (Block.cpp:128-133)
        const int sbRow = b.r & sbMask, sbCol = b.c & sbMask;
        for (int plane = 0; plane < 1 + b.has_chroma * 2; plane++) {
            const int psz = plane ? av1r_ss420[b.bsize] : b.bsize;
            const int sub = plane ? 1 : 0;
            if (flag(plane, (sbRow >> sub) - 1, (sbCol >> sub) + bw4_of(psz))) rec.ii_edge |= (uint8_t)(1 << (2 * plane));
            if (flag(plane, (sbRow >> sub) + bh4_of(psz), (sbCol >> sub) - 1)) rec.ii_edge |= (uint8_t)(2 << (2 * plane));
        }
    }
    if (b.pal_y || b.pal_uv) {
        rec.palette_off = (uint32_t)F.palette.size();
        uint8_t hdr[AV1R_PALETTE_HDR];
        memset(hdr, 0, sizeof(hdr));
        hdr[0] = (uint8_t)(b.pal_y ? b.map_wy : 0);
        hdr[1] = (uint8_t)(b.pal_y ? b.map_hy : 0);
        hdr[2] = (uint8_t)(b.pal_uv ? b.map_wuv : 0);
        hdr[3] = (uint8_t)(b.pal_uv ? b.map_huv : 0);
        for (int i = 0; i < 8; i++) {
            if (i < b.pal_y) hdr[4 + i] = b.colors[0][i];
            if (i < b.pal_uv) {
                hdr[12 + i] = b.colors[1][i];
                hdr[20 + i] = b.colors[2][i];
            }
        }
        F.palette.insert(F.palette.end(), hdr, hdr + AV1R_PALETTE_HDR);
        if (b.pal_y) F.palette.insert(F.palette.end(), b.map_y.begin(), b.map_y.end());
        if (b.pal_uv) F.palette.insert(F.palette.end(), b.map_uv.begin(), b.map_uv.end());
        while (F.palette.size() & 3) F.palette.push_back(0);
    }
    if (b.is_inter && b.motion_mode == LOCALWARP) {
        warp_estimation(b);
        if (b.local_valid) {
            f |= AV1R_BLK_LOCAL_VALID;
            memcpy(rec.local_warp, b.local_warp, sizeof(rec.local_warp));
        }
    }
    rec.flags = f;
    rec.first_tb = (uint32_t)F.tbs.size();
    int maxLumaW = 0, maxLumaH = 0;
    for (const Tb& t : tbs) {
        const int plane = t.plane, sub = plane ? 1 : 0;
        const int row = (t.y << sub) >> 2, col = (t.x << sub) >> 2;
        const int sbRow = row & sbMask, sbCol = col & sbMask;
        const int stepX = av1r_tx_w[t.tx] >> 2, stepY = av1r_tx_h[t.tx] >> 2;
        F.tbs.emplace_back();  // (zeroed)
        av1r_tb& tr = F.tbs.back();
        tr.block = blockIdx;
        tr.x = (uint16_t)t.x;
        tr.y = (uint16_t)t.y;
        tr.plane = (uint8_t)plane;
        tr.tx_size = (uint8_t)t.tx;
        tr.tx_type = (uint8_t)(t.eob ? t.type : 0);
        const bool haveL = (plane == 0 ? b.avail_l : b.avail_l_uv) || t.x > t.base_x;
        const bool haveA = (plane == 0 ? b.avail_u : b.avail_u_uv) || t.y > t.base_y;
        const bool haveAR = flag(plane, (sbRow >> sub) - 1, (sbCol >> sub) + stepX);
        const bool haveBL = flag(plane, (sbRow >> sub) + stepY, (sbCol >> sub) - 1);
        tr.flags = (uint8_t)((haveL ? AV1R_TB_HAVE_LEFT : 0) | (haveA ? AV1R_TB_HAVE_ABOVE : 0) |
                             (haveAR ? AV1R_TB_HAVE_AR : 0) | (haveBL ? AV1R_TB_HAVE_BL : 0));
        tr.coef_off = t.coef_off;
        tr.coef_cnt = (uint16_t)t.coef_cnt;
        if (plane && !b.is_inter) {
            rec.max_luma_w = (uint16_t)maxLumaW;
            rec.max_luma_h = (uint16_t)maxLumaH;
        }
        // TransformBlock::decode side effects (TransformBlock.cpp:2418-2454)
        if (!b.is_inter && plane == 0) {
            maxLumaW = t.x + stepX * 4;
            maxLumaH = t.y + stepY * 4;
        }
        for (int i = 0; i < stepY; i++)
            for (int j = 0; j < stepX; j++) {
                // (the loop filter's transform sizes: only the emitted mode-info grid reads them)
                if (P.emit_mi)
                    for (int xx = 0; xx <= sub; xx++)
                        for (int yy = 0; yy <= sub; yy++) {
                            const int rr = row + (i << sub) + yy, cc = col + (j << sub) + xx;
                            if (rr < fh.aligned_mi_rows && cc < fh.aligned_mi_cols) P.mi_lftx[((size_t)rr * P.mi_stride + cc) * 3 + plane] = (uint8_t)t.tx;
                        }
                T.decoded[plane][(sbRow >> sub) + i + 1][(sbCol >> sub) + j + 1] = 1;
            }
    }
    rec.n_tbs = (uint32_t)F.tbs.size() - rec.first_tb;
}

// ------------------------------------------------------------------------------------
// loop restoration syntax (Parser.cpp:2112-2225)
// ------------------------------------------------------------------------------------
static int decode_subexp_bool(SymbolDecoder& sd, int numSyms, int k)
{
    int i = 0, mk = 0;
    for (;;) {
        const int b2 = i ? k + i - 1 : k;
        const int a = 1 << b2;
        if (numSyms <= mk + 3 * a) return (int)sd.ns((uint32_t)(numSyms - mk)) + mk;
        if (sd.literal(1)) {
            i++;
            mk += a;
        } else {
            return (int)sd.literal(b2) + mk;
        }
    }
}
static int inverse_recenter(int r, int v)
{
    if (v > 2 * r) return v;
    if (v & 1) return r - ((v + 1) >> 1);
    return r + (v >> 1);
}
static int decode_signed_subexp_with_ref_bool(SymbolDecoder& sd, int low, int high, int k, int r)
{
    const int mx = high - low;
    r -= low;
    const int v = decode_subexp_bool(sd, mx, k);
    const int x = (r << 1) <= mx ? inverse_recenter(r, v) : mx - 1 - inverse_recenter(mx - 1 - r, v);
    return x + low;
}

void BlockParser::read_lr(int r, int c, int bsize)
{
    if (fh.allow_intrabc) return;
    const int w = bw4_of(bsize), h = bh4_of(bsize);
    for (int plane = 0; plane < 3; plane++) {
        if (!fh.uses_lr || fh.lr_type[plane] == AV1R_RESTORE_NONE) continue;
        const int sub = plane ? 1 : 0;
        const int unitSize = fh.lr_unit_size[plane];
        const int rowStart = (r * (4 >> sub) + unitSize - 1) / unitSize;
        const int rowEnd = std::min(fh.lr_unit_rows[plane], ((r + h) * (4 >> sub) + unitSize - 1) / unitSize);
        const int num = 4 >> sub, den = unitSize;
        const int colStart = (c * num + den - 1) / den;
        const int colEnd = std::min(fh.lr_unit_cols[plane], ((c + w) * num + den - 1) / den);
        for (int ur = rowStart; ur < rowEnd; ur++)
            for (int uc = colStart; uc < colEnd; uc++) {
                av1r_lr_unit& u = P.lr_units[P.lr_off[plane] + (size_t)ur * fh.lr_unit_cols[plane] + uc];
                int type;
                if (fh.lr_type[plane] == AV1R_RESTORE_WIENER)
                    type = S(cdf.mode.wiener_restore, 2) ? AV1R_RESTORE_WIENER : AV1R_RESTORE_NONE;
                else if (fh.lr_type[plane] == AV1R_RESTORE_SGRPROJ)
                    type = S(cdf.mode.sgrproj_restore, 2) ? AV1R_RESTORE_SGRPROJ : AV1R_RESTORE_NONE;
                else
                    type = S(cdf.mode.switchable_restore, 3);
                u.type = (uint8_t)type;
                if (type == AV1R_RESTORE_WIENER) {
                    for (int pass = 0; pass < 2; pass++) {
                        const int first = plane ? 1 : 0;
                        if (plane) u.wiener[pass][0] = 0;
                        for (int j = first; j < 3; j++) {
                            const int v = decode_signed_subexp_with_ref_bool(sd, kWienerTapsMin[j], kWienerTapsMax[j] + 1,
                                                                             kWienerTapsK[j], T.ref_lr_wiener[plane][pass][j]);
                            u.wiener[pass][j] = (int8_t)v;
                            T.ref_lr_wiener[plane][pass][j] = v;
                        }
                    }
                } else if (type == AV1R_RESTORE_SGRPROJ) {
                    const int set = (int)L(4);
                    u.sgr_set = (uint8_t)set;
                    for (int i = 0; i < 2; i++) {
                        const int radius = av1r_sgr_params[set][i * 2];
                        int v;
                        if (radius) {
                            v = decode_signed_subexp_with_ref_bool(sd, kSgrprojXqdMin[i], kSgrprojXqdMax[i] + 1, 4,
                                                                   T.ref_sgr_xqd[plane][i]);
                        } else {
                            v = 0;
                            if (i == 1) v = clip3(kSgrprojXqdMin[i], kSgrprojXqdMax[i], (1 << 7) - T.ref_sgr_xqd[plane][0]);
                        }
                        u.sgr_xqd[i] = (int8_t)v;
                        T.ref_sgr_xqd[plane][i] = v;
                    }
                }
            }
    }
}

}  // namespace

// ------------------------------------------------------------------------------------
// tile (Tile::parse, Tile.cpp:122-160; BlockDecoded, Tile.cpp:41-90)
// ------------------------------------------------------------------------------------
void TileCtx::clear_block_decoded_flags(int r, int c, int sbSize4)
{
    for (int plane = 0; plane < 3; plane++) {
        const int sub = plane ? 1 : 0;
        const int sbWidth4 = (mi_col_end - c) >> sub, sbHeight4 = (mi_row_end - r) >> sub;
        memset(decoded[plane], 0, sizeof(decoded[plane]));
        for (int y = -1; y <= (sbSize4 >> sub); y++)
            for (int x = -1; x <= (sbSize4 >> sub); x++) {
                const bool on = (y < 0 && x < sbWidth4) || (!(y < 0 && x < sbWidth4) && x < 0 && y < sbHeight4);
                decoded[plane][y + 1][x + 1] = on;
            }
        decoded[plane][(sbSize4 >> sub) + 1][0] = 0;
    }
}

int Parser::decode_tile(TileCtx& T)
{
    const int sbSize = seq.use_128x128 ? BLOCK_128X128 : BLOCK_64X64;
    const int sbSize4 = av1r_num4x4w[sbSize];
    for (int p = 0; p < 3; p++) {
        T.above_level[p].assign(fh.aligned_mi_cols + 32, 0);
        T.above_dc[p].assign(fh.aligned_mi_cols + 32, 0);
    }
    for (int i = 0; i < 4; i++) T.delta_lf[i] = 0;
    for (int plane = 0; plane < 3; plane++)
        for (int pass = 0; pass < 2; pass++) {
            T.ref_sgr_xqd[plane][pass] = kSgrprojXqdMid[pass];
            for (int i = 0; i < 3; i++) T.ref_lr_wiener[plane][pass][i] = kWienerTapsMid[i];
        }
    BlockParser bp(*this, T);
    for (int r = T.mi_row_start; r < T.mi_row_end; r += sbSize4) {
        for (int p = 0; p < 3; p++) {
            T.left_level[p].assign(fh.aligned_mi_rows + 32, 0);
            T.left_dc[p].assign(fh.aligned_mi_rows + 32, 0);
        }
        for (int c = T.mi_col_start; c < T.mi_col_end; c += sbSize4) {
            T.read_deltas = fh.delta_q_present;
            T.clear_block_decoded_flags(r, c, sbSize4);
            bp.read_lr(r, c, sbSize);
            bp.decode_partition(r, c, sbSize);
            if (!T.err.empty()) return AV1R_E_INVALID;
        }
    }
    return AV1R_OK;
}

}  // namespace av1p
