// av1p.h -- host AV1 parser: OBUs -> av1r frame batches (include/av1r.h).
//
// The reference decoder's parse half (oddstone/av1dec: decoder/Parser.cpp, BitReader.cpp,
// SymbolDecoder.cpp, EntropyDecoder.cpp, Tile.cpp, Partition.cpp, Block.cpp:313-2271,
// TransformBlock.cpp:1165-1705, InterPredict.cpp:1051-1671) rebuilt as a flat, allocation
// free C++ pipeline.  Instead of a SuperBlock -> Partition -> Block -> TransformBlock object
// tree per frame (37 KB per TransformBlock, Block.cpp:193), the parser writes the device
// batch directly: block and transform-block records in decode order, packed non-zero
// coefficients, the per-4x4 mode-info grid, palette maps, CDEF indices and loop
// restoration units, plus the per-block values reconstruction needs from the decode-time
// state of the reference (edge availability, local warp parameters, MaxLumaW/H).
//
// Everything follows the AV1 specification's syntax and semantics; the reference's
// behaviour is matched where it is defined (its undefined behaviour -- out-of-range reads,
// K5 in SURVEY.md -- is not reproduced).  Segmentation features, superres, film-grain
// synthesis, >8-bit and non-4:2:0 are outside the reference's support and are rejected
// with AV1R_E_UNSUPPORTED.
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "av1r.h"
#include "av1r_consts.h"
#include "cdf_default.h"

namespace av1p {

// ---- enumerations (numeric values of the reference's aom/enums.h) ----
enum { KEY_FRAME = 0, INTER_FRAME = 1, INTRA_ONLY_FRAME = 2, SWITCH_FRAME = 3 };
enum { NONE_FRAME = -1, INTRA_FRAME = 0, LAST_FRAME = 1, LAST2_FRAME, LAST3_FRAME, GOLDEN_FRAME, BWDREF_FRAME, ALTREF2_FRAME,
       ALTREF_FRAME };
enum { PARTITION_NONE, PARTITION_HORZ, PARTITION_VERT, PARTITION_SPLIT, PARTITION_HORZ_A, PARTITION_HORZ_B, PARTITION_VERT_A,
       PARTITION_VERT_B, PARTITION_HORZ_4, PARTITION_VERT_4 };
enum { TX_MODE_ONLY_4X4, TX_MODE_LARGEST, TX_MODE_SELECT };
enum { OBU_SEQUENCE_HEADER = 1, OBU_TEMPORAL_DELIMITER = 2, OBU_FRAME_HEADER = 3, OBU_TILE_GROUP = 4, OBU_METADATA = 5,
       OBU_FRAME = 6, OBU_REDUNDANT_FRAME_HEADER = 7, OBU_TILE_LIST = 8, OBU_PADDING = 15 };
enum { SWITCHABLE = 4 };
enum { TX_SET_DCTONLY = 0, TX_SET_1 = 1, TX_SET_2 = 2, TX_SET_3 = 3 };
enum { TX_CLASS_2D = 0, TX_CLASS_HORIZ = 1, TX_CLASS_VERT = 2 };

constexpr int kNumRefFrames = 8;
constexpr int kRefsPerFrame = 7;
constexpr int kPrimaryRefNone = 7;
constexpr int kWarpPrecBits = 16;
constexpr int kMaxRefMvStack = 8;
constexpr int kRefCatLevel = 640;
constexpr int kMvBorder = 128;  // MV_BORDER (16 pel, 1/8 units)

struct Mv {
    int16_t r = 0, c = 0;
    bool operator==(const Mv& o) const { return r == o.r && c == o.c; }
};

// ---- bit reader (OBU / header syntax, MSB first) ----
struct BitReader {
    const uint8_t* d = nullptr;
    size_t n = 0;      // bytes
    size_t pos = 0;    // bits consumed
    bool over = false; // read past the end
    BitReader() = default;
    BitReader(const uint8_t* p, size_t sz) : d(p), n(sz) {}
    uint32_t f(int bits)
    {
        uint32_t v = 0;
        for (int i = 0; i < bits; i++) {
            const size_t byte = pos >> 3;
            uint32_t b = 0;
            if (byte < n) b = (d[byte] >> (7 - (pos & 7))) & 1;
            else over = true;
            v = (v << 1) | b;
            pos++;
        }
        return v;
    }
    bool flag() { return f(1) != 0; }
    int su(int bits)  // su(n)
    {
        int v = (int)f(bits);
        const int signMask = 1 << (bits - 1);
        if (v & signMask) v -= 2 * signMask;
        return v;
    }
    uint32_t ns(uint32_t nv)  // ns(n)
    {
        int w = 0;
        for (uint32_t x = nv; x; x >>= 1) w++;
        const uint32_t m = (1u << w) - nv;
        const uint32_t v = f(w - 1);
        if (v < m) return v;
        return (v << 1) - m + f(1);
    }
    uint32_t uvlc()
    {
        int lz = 0;
        while (!over && !f(1)) lz++;
        if (lz >= 32) return UINT32_MAX;
        return f(lz) + ((1u << lz) - 1);
    }
    uint64_t leb128()
    {
        uint64_t v = 0;
        for (int i = 0; i < 8; i++) {
            const uint32_t b = f(8);
            v |= (uint64_t)(b & 0x7f) << (i * 7);
            if (!(b & 0x80)) break;
        }
        return v;
    }
    uint32_t le(int bytes)
    {
        uint32_t t = 0;
        for (int i = 0; i < bytes; i++) t += f(8) << (i * 8);
        return t;
    }
    void byte_align() { pos = (pos + 7) & ~(size_t)7; }
    size_t byte_pos() const { return pos >> 3; }
};

#ifdef AV1P_WRITER
// Bitstream-writer build only (tools/bsw): the symbol reads of the syntax walk are answered by
// a chooser that also arithmetic-codes the chosen symbol, so the same walk writes a stream.
struct WriterHook {
    virtual int symbol(uint16_t* cdf, int nsym) = 0;  // choose a value and encode it
    virtual void mv_pred(const Mv& pred, int ctx) = 0;  // read_mv: the predictor of the next vector
    virtual void golomb_prefix(int length) = 0;         // the next literal bit is Golomb prefix bit `length`
    virtual ~WriterHook() {}
};
#endif

// ---- arithmetic decoder (AV1 spec 8.2: init_symbol / read_symbol / exit_symbol) with
// CDFs in libaom's inverted form (32768 - cumulative, then the adaptation counter) ----
struct SymbolDecoder {
    // The decoder state in the windowed form (the spec's SymbolValue with the following bits
    // of the tile already shifted in, complemented: libaom's od_ec_dec, which the reference's
    // SymbolDecoder also uses): the top 16 bits of `dif` compare against the interval
    // boundaries; bytes are XORed in 8 at a time when `cnt` runs out, so a symbol costs no
    // per-bit refill.  Past the end of the tile the data reads as zero bits (spec 8.2.2).
    const uint8_t* p = nullptr;
    const uint8_t* end = nullptr;
    uint64_t dif = 0;
    uint32_t range = 0;  // SymbolRange
    int cnt = 0;
    bool noUpdate = false;

    void refill()
    {
        int sh = 64 - 9 - (cnt + 15);
        if (end - p >= 8 && sh >= 0) {
            // 8 bytes at once (big-endian): byte k to shift sh - 8k, for the nb bytes that fit
            // whole (the next byte's bits below the last one's are masked off)
            uint64_t w;
            memcpy(&w, p, 8);
            w = __builtin_bswap64(w);
            const int nb = (sh >> 3) + 1, lo = sh - 8 * (nb - 1);
            dif ^= (w >> (56 - sh)) & ~((1ull << lo) - 1);
            cnt += 8 * nb;
            p += nb;
            return;
        }
        for (; sh >= 0 && p < end; sh -= 8, p++) {
            dif ^= (uint64_t)*p << sh;
            cnt += 8;
        }
        if (p >= end) cnt = 0x4000;  // zeros (ones in dif) from here on: never refill again
    }
    void init(const uint8_t* data, size_t sz, bool disableCdfUpdate)
    {
        p = data;
        end = data + sz;
        dif = ((uint64_t)1 << 63) - 1;
        range = 0x8000;
        cnt = -15;
        refill();
        noUpdate = disableCdfUpdate;
    }
    void renorm(uint64_t d64)
    {
        const int d = __builtin_clz(range) - 16;  // 15 - FloorLog2(range)
        cnt -= d;
        dif = ((d64 + 1) << d) - 1;
        range <<= d;
        if (cnt < 0) refill();
    }
#ifdef AV1P_WRITER
    WriterHook* hook = nullptr;
#endif
    int read(uint16_t* cdf, int nsym)
    {
#ifdef AV1P_TRACE
        const uint32_t range0 = range;
        uint16_t cdf0[16];
        for (int q = 0; q < nsym; q++) cdf0[q] = cdf[q];
#endif
#ifdef AV1P_WRITER
        if (hook) {
            const int s = hook->symbol(cdf, nsym);
            if (!noUpdate) adapt(cdf, s, nsym);
            return s;
        }
#endif
#if !defined(AV1P_WRITER) && !defined(AV1P_TRACE) && !defined(AV1P_READ_LOOP)
        // the alphabets the syntax uses, each as readN (branch-free interval search, unrolled
        // adaptation): the loop below mispredicts once per symbol on the larger ones
        switch (nsym) {
        case 2: return readN<2>(cdf);
        case 3: return readN<3>(cdf);
        case 4: return readN<4>(cdf);
        case 5: return readN<5>(cdf);
        case 6: return readN<6>(cdf);
        case 7: return readN<7>(cdf);
        case 8: return readN<8>(cdf);
        case 9: return readN<9>(cdf);
        case 10: return readN<10>(cdf);
        case 11: return readN<11>(cdf);
        case 12: return readN<12>(cdf);
        case 13: return readN<13>(cdf);
        case 14: return readN<14>(cdf);
        case 15: return readN<15>(cdf);
        case 16: return readN<16>(cdf);
        default: break;
        }
#endif
        const uint32_t c = (uint32_t)(dif >> 48);
        uint32_t cur = range, prev;
        int sym = -1;
        do {
            sym++;
            prev = cur;
            cur = ((range >> 8) * (uint32_t)(cdf[sym] >> 6) >> 1) + 4u * (uint32_t)(nsym - sym - 1);
        } while (c < cur);
        range = prev - cur;
        renorm(dif - ((uint64_t)cur << 48));
        if (!noUpdate) adapt(cdf, sym, nsym);
#ifdef AV1P_TRACE  // debug aid: the symbol sequence, for diffing against another decoder
        {
            static FILE* tf = fopen("/tmp/av1p_sym.txt", "w");
            fprintf(tf, "%d %d %u", nsym, sym, range0);
            for (int q = 0; q < nsym; q++) fprintf(tf, " %u", cdf0[q]);
            fprintf(tf, "\n");
        }
#endif
        return sym;
    }
    // read() with the alphabet size known at compile time, always inlined: the coefficient
    // loop's symbols (2-4 symbol alphabets, ~60 % of a frame's symbols) without a call, with
    // the interval search and the adaptation unrolled.  Same arithmetic as read().
    template <int N>
    __attribute__((always_inline)) int readN(uint16_t* cdf)
    {
#if defined(AV1P_WRITER) || defined(AV1P_TRACE)
        return read(cdf, N);
#else
        const uint32_t c = (uint32_t)(dif >> 48);
        const uint32_t r8 = range >> 8;
        uint32_t v[N + 1];
        v[0] = range;
#pragma GCC unroll 16
        for (int i = 0; i < N - 1; i++) v[i + 1] = (r8 * (uint32_t)(cdf[i] >> 6) >> 1) + 4u * (uint32_t)(N - i - 1);
        v[N] = 0;
        int sym = 0;
#pragma GCC unroll 16
        for (int i = 1; i < N; i++) sym += c < v[i];  // the boundaries fall with i
        range = v[sym] - v[sym + 1];
        renorm(dif - ((uint64_t)v[sym + 1] << 48));
        if (!noUpdate) {
            const int cnt = cdf[N];
            const int rate = 3 + (cnt > 15) + (cnt > 31) + (N >= 4 ? 2 : N >= 2 ? 1 : 0);
            // branch-free: the symbol decides the direction of every entry, and a branch on
            // it mispredicts as often as the symbol changes
#pragma GCC unroll 16
            for (int i = 0; i < N - 1; i++) {
                const uint32_t m = 0u - (uint32_t)(i < sym);
                const uint32_t up = (32768u - cdf[i]) >> rate, dn = (uint32_t)cdf[i] >> rate;
                cdf[i] = (uint16_t)(cdf[i] + ((up & m) - (dn & ~m)));
            }
            cdf[N] += cdf[N] < 32;
        }
        return sym;
#endif
    }
    static void adapt(uint16_t* cdf, int sym, int nsym)
    {
        const int cnt = cdf[nsym];
        const int rate = 3 + (cnt > 15) + (cnt > 31) + (nsym >= 4 ? 2 : nsym >= 2 ? 1 : 0);
        // below the symbol the (inverted) CDF moves up toward 32768, from it on down toward 0
        // (the spec's single loop with tmp = 32768 / 0, as two branch-free runs)
        for (int i = 0; i < sym; i++) cdf[i] += (uint16_t)((32768u - cdf[i]) >> rate);
        for (int i = sym; i < nsym - 1; i++) cdf[i] -= (uint16_t)(cdf[i] >> rate);
        cdf[nsym] += cdf[nsym] < 32;
    }
    int boolean()  // read_literal bit: probability 1/2, never adapted
    {
#if !defined(AV1P_WRITER) && !defined(AV1P_TRACE)
        // read() over the CDF {16384, 0}: the first interval boundary, then the same renormalisation
        // (selects, not a branch: these bits are close to random)
        const uint32_t v0 = ((range >> 8) << 7) + 4;
        const bool one = (uint32_t)(dif >> 48) < v0;
        range = one ? v0 : range - v0;
        renorm(one ? dif : dif - ((uint64_t)v0 << 48));
        return one;
#endif
        uint16_t c[3] = {16384, 0, 0};
        const bool nu = noUpdate;
        noUpdate = true;
        const int v = read(c, 2);
        noUpdate = nu;
        return v;
    }
    uint32_t literal(int n)
    {
        uint32_t x = 0;
        for (int i = 0; i < n; i++) x = 2 * x + boolean();
        return x;
    }
    uint32_t ns(uint32_t nv)
    {
        int w = 0;
        for (uint32_t x = nv; x; x >>= 1) w++;
        const uint32_t m = (1u << w) - nv;
        const uint32_t v = literal(w - 1);
        if (v < m) return v;
        return (v << 1) - m + literal(1);
    }
};

struct Cdfs {
    CoefCdfs coef;
    ModeCdfs mode;
    MvCdfs mv[2];
    void reset_counters();
};

// ---- sequence header (spec 5.5) ----
struct SeqHdr {
    int profile = 0;
    bool still_picture = false, reduced_still_picture_header = false;
    bool timing_info_present = false, decoder_model_info_present = false, equal_picture_interval = false;
    int buffer_delay_length = 0, buffer_removal_time_length = 0, frame_presentation_time_length = 0;
    int operating_points = 1;
    int op_idc[32] = {};
    bool decoder_model_present_for_op[32] = {};
    int frame_width_bits = 0, frame_height_bits = 0, max_frame_width = 0, max_frame_height = 0;
    bool frame_id_numbers_present = false;
    int delta_frame_id_length = 0, additional_frame_id_length = 0;
    bool use_128x128 = false, enable_filter_intra = false, enable_intra_edge_filter = false;
    bool enable_interintra_compound = false, enable_masked_compound = false, enable_warped_motion = false;
    bool enable_dual_filter = false, enable_order_hint = false, enable_jnt_comp = false, enable_ref_frame_mvs = false;
    int seq_force_screen_content_tools = 2, seq_force_integer_mv = 2;
    int order_hint_bits = 0;
    bool enable_superres = false, enable_cdef = false, enable_restoration = false;
    int bit_depth = 8;
    bool mono_chrome = false, subx = true, suby = true;
    bool separate_uv_delta_q = false;
    bool film_grain_params_present = false;
    int num_planes = 3;
};

// ---- per reference slot: what later frames load (spec 7.20 / 7.21) ----
struct RefSlot {
    bool valid = false;
    int frame_id = 0;
    int upscaled_width = 0, frame_width = 0, frame_height = 0, render_width = 0, render_height = 0;
    int mi_cols = 0, mi_rows = 0;
    int frame_type = 0;
    int order_hint = 0;
    int saved_order_hints[8] = {};
    int32_t saved_gm[8][6] = {};
    int8_t lf_ref_deltas[8] = {}, lf_mode_deltas[2] = {};
    std::vector<int8_t> mf_ref;  // MfRefFrames at (2 y8 + 1, 2 x8 + 1), (mi_rows / 2) x (mi_cols / 2)
    std::vector<Mv> mf_mv;       // MfMvs
    Cdfs cdfs;
    bool showable = false;
};

// ---- per 4x4 parse state of the current frame (ModeInfoBlock, Parser.h:432-455) ----
struct MiInfo {
    Mv mv[2];
    int8_t ref[2];
    uint8_t mi_size, y_mode, uv_mode;
    uint8_t is_inter, skip, skip_mode;
    uint8_t inter_tx, tx_type;
    uint8_t interp[2];
    uint8_t comp_group_idx, compound_idx;
    uint8_t pal_size[2];
    uint8_t pad[4];
    uint32_t pal_idx;  // this block's palette colours (Parser::pal_colors), ~0u: none
};
// (32 bytes: two per cache line, none straddling one; the loop filter's transform sizes and
// delta LF live in Parser::mi_lftx / mi_dlf, filled only for an emitted mode-info grid)
static_assert(sizeof(MiInfo) == 32, "MiInfo layout");

// ---- frame header (spec 5.9 uncompressed_header) and everything derived from it ----
struct FrameHdr {
    bool show_existing_frame = false;
    int frame_to_show = 0;
    int frame_type = 0;
    bool frame_is_intra = false, show_frame = false, showable_frame = false, error_resilient = false;
    bool disable_cdf_update = false, allow_screen_content_tools = false, force_integer_mv = false;
    int current_frame_id = 0;
    bool frame_size_override = false;
    int order_hint = 0;
    int primary_ref_frame = kPrimaryRefNone;
    int refresh_frame_flags = 0;
    int frame_width = 0, frame_height = 0, upscaled_width = 0, render_width = 0, render_height = 0;
    bool use_superres = false;
    int superres_denom = 8;
    int mi_cols = 0, mi_rows = 0, aligned_mi_cols = 0, aligned_mi_rows = 0;
    bool allow_intrabc = false;
    int ref_frame_idx[7] = {};
    bool allow_high_precision_mv = false, is_motion_mode_switchable = false, use_ref_frame_mvs = false;
    int interpolation_filter = 0;
    int order_hints[8] = {};
    bool ref_frame_sign_bias[8] = {};
    bool disable_frame_end_update_cdf = true;
    // tiles
    int tile_cols = 1, tile_rows = 1, tile_cols_log2 = 0, tile_rows_log2 = 0;
    std::vector<int> mi_col_starts, mi_row_starts;
    int context_update_tile_id = 0, tile_size_bytes = 4;
    // quantizer
    int base_q_idx = 0;
    int delta_q_y_dc = 0, delta_q_u_dc = 0, delta_q_u_ac = 0, delta_q_v_dc = 0, delta_q_v_ac = 0;
    bool using_qmatrix = false;
    bool segmentation_enabled = false;
    bool delta_q_present = false, delta_lf_present = false, delta_lf_multi = false;
    int delta_q_res = 0, delta_lf_res = 0;
    bool coded_lossless = false, all_lossless = false;
    // loop filter
    int lf_level[4] = {}, lf_sharpness = 0;
    bool lf_delta_enabled = false;
    int8_t lf_ref_deltas[8] = {}, lf_mode_deltas[2] = {};
    // cdef
    int cdef_damping = 3, cdef_bits = 0;
    int cdef_y_pri[8] = {}, cdef_y_sec[8] = {}, cdef_uv_pri[8] = {}, cdef_uv_sec[8] = {};
    // loop restoration
    bool uses_lr = false;
    int lr_type[3] = {}, lr_unit_size[3] = {}, lr_unit_rows[3] = {}, lr_unit_cols[3] = {};
    int tx_mode = 0;
    bool reference_select = false, skip_mode_present = false;
    int skip_mode_frame[2] = {};
    bool allow_warped_motion = false, reduced_tx_set = false;
    int gm_type[8] = {};
    int32_t gm_params[8][6] = {};
    int32_t prev_gm[8][6] = {};
};

struct Frame;  // one decoded frame's batch (api.cpp)

// Everything one tile's parse owns (Tile::parse, Tile.cpp:122-160): its entropy decoder and
// CDFs, the above / left contexts, the per-tile delta and loop-restoration references, and
// the records it emits.  Tiles are independent for entropy decoding and read only their own
// region of the mode-info grid (every neighbour test is bounded by the tile), so the tiles of
// a frame parse concurrently, one TileCtx each, and are merged into the frame in tile order
// (Parser::merge_tile fixes the record indices).
struct TileCtx {
    int mi_row_start = 0, mi_row_end = 0, mi_col_start = 0, mi_col_end = 0;
    SymbolDecoder sd;
    Cdfs tcdf;  // the tile's CDFs
    // level contexts are int16 as the reference's BlockContext::LevelContext: a Golomb level
    // past int16 wraps negative and stays so in the context (TransformBlock.cpp:1620-1702)
    std::vector<int16_t> above_level[3], left_level[3];
    std::vector<uint8_t> above_dc[3], left_dc[3];
    int delta_lf[4] = {};
    int current_q = 0;
    bool read_deltas = false;
    int ref_sgr_xqd[3][2] = {};
    int ref_lr_wiener[3][2][3] = {};
    // decoded flags of the current superblock (Tile.cpp BlockDecoded), per plane, offset 1
    static constexpr int kDecN = 35;
    uint8_t decoded[3][kDecN][kDecN] = {};
    std::vector<std::vector<uint8_t>> pal_colors;  // per palette block: 24 colours (y, u, v)
    // this tile's records; block.first_tb / palette_off and tb.block / coef_off are
    // tile-relative until the tile is merged into the frame
    std::vector<av1r_block> blocks;
    std::vector<av1r_tb> tbs;
    std::vector<uint32_t> coefs;
    std::vector<uint8_t> palette;
    std::string err;
    int fail(int code, const char* fmt, ...);
    bool is_inside(int r, int c) const
    {
        return c >= mi_col_start && c < mi_col_end && r >= mi_row_start && r < mi_row_end;
    }
    void clear_block_decoded_flags(int r, int c, int sbSize4);
};

class Parser {
public:
    Parser();
    // one temporal unit of OBUs (Decoder::decode, Av1Decoder.cpp:49-109); completed frames
    // (decoded or shown-existing) are appended to `out` as batches
    int decode_tu(const uint8_t* data, size_t size);
    std::vector<Frame*> done;  // frames completed by the last decode_tu (owned by the caller)
    std::string err;
    int fail(int code, const char* fmt, ...);

    // ---- state ----
    SeqHdr seq;
    bool have_seq = false;
    FrameHdr fh;
    bool seen_frame_header = false;
    RefSlot slots[8];
    Cdfs cdf;        // the frame's CDFs (init / load at header time)
    Cdfs saved_cdf;  // the context_update_tile_id tile's CDFs at its end
    int tile_num = 0;
    // per frame
    std::vector<MiInfo> mi;
    int mi_stride = 0;
    // per 4x4 unit, for the emitted grid only (emit_mi): lf_tx of the 3 planes, delta LF x 4
    std::vector<uint8_t> mi_lftx;
    std::vector<int8_t> mi_dlf;
    std::vector<int8_t> mf_ref;          // MfRefFrames of this frame (motion vector storage), per 8x8
    std::vector<Mv> mf_mv;
    std::vector<Mv> motion_field[8];     // MotionFieldMvs[ref][row >> 1][col >> 1]
    std::vector<int8_t> cdef_idx;        // per 64x64 (frame cdef grid)
    int cdef_cols = 0, cdef_rows = 0;
    std::vector<av1r_lr_unit> lr_units;  // frame order: plane 0 units, plane 1, plane 2
    int lr_off[3] = {};
    Frame* cur = nullptr;
    // frames handed back by av1p_decode_tu's next call, reused with their vectors' capacity
    // (a 1080p frame's records grow to ~3 MB: no reallocation and first-touch faults per frame)
    std::vector<Frame*> spare;
    Frame* take_frame();

    // ---- per tile ----
    TileCtx tile;  // the serial path's tile (and the bitstream writer's)
    // tile-parallel parsing: up to `tile_threads` threads parse the tiles of a tile group
    // (1: serial); one TileCtx per tile, kept between frames for their buffers
    int tile_threads = 1;
    // fill the batch's per-4x4 mode-info grid (av1p_set_mode_info)
    bool emit_mi = true;
    std::vector<TileCtx*> par_tiles;
    ~Parser();

    // ---- obu.cpp ----
    int parse_sequence_header(BitReader& br);
    int parse_frame_header(BitReader& br);
    int parse_uncompressed_header(BitReader& br);
    int frame_size(BitReader& br);
    int superres_params(BitReader& br);
    void compute_image_size();
    int render_size(BitReader& br);
    int frame_size_with_refs(BitReader& br);
    void set_frame_refs(int last_idx, int gold_idx);
    int tile_info(BitReader& br);
    int read_delta_q(BitReader& br);
    int global_motion_params(BitReader& br);
    int film_grain_params(BitReader& br);
    void setup_past_independence();
    void load_previous();
    int skip_mode_params(BitReader& br);
    int relative_dist(int a, int b) const;
    void motion_field_estimation();
    bool mv_project(int src, int dstSign);
    int tile_group(BitReader& br, const uint8_t* data, size_t size);
    void start_frame();
    int finish_frame();
    void reference_update();
    void show_existing();
    void fill_header(av1r_frame_hdr& o) const;

    // tile `tn` of the frame over `size` bytes at `data`: T's bounds, CDFs, decoder, outputs
    void begin_tile(TileCtx& T, int tn, const uint8_t* data, size_t size);
    // T's records appended to the frame (indices made frame-relative), its CDFs saved when it
    // is the context_update_tile_id tile, its error reported
    int merge_tile(TileCtx& T, int tn);

    // ---- block.cpp (the block-level syntax lives in its BlockParser) ----
    int decode_tile(TileCtx& T);
    MiInfo& mi_at(int r, int c) { return mi[(size_t)r * mi_stride + c]; }
};

// frame batch storage (api.cpp): the arrays an av1r_frame_batch points into
struct Frame {
    av1r_frame_hdr hdr;
    std::vector<av1r_mi> mi;
    std::vector<av1r_block> blocks;
    std::vector<av1r_tb> tbs;
    std::vector<uint32_t> coefs;
    std::vector<uint8_t> palette;
    std::vector<int8_t> cdef;
    std::vector<av1r_lr_unit> lr;
    av1r_frame_batch batch;
    void bind();
};

}  // namespace av1p
