// obu.cpp -- OBU, sequence-header and frame-header syntax, reference management and the
// frame-level driver of the host parser (AV1 spec 5.3-5.12, 7.5-7.21).
//
// Reference behaviour restated (oddstone/av1dec):
//   Decoder::decode OBU loop           decoder/Av1Decoder.cpp:49-109
//   SequenceHeader::parse              decoder/Parser.cpp:142-436
//   FrameHeader::parse                 decoder/Parser.cpp:1152-1403
//   tile info / quant / LF / CDEF / LR decoder/Parser.cpp:1563-1643, 1733-1760, 1874-2111
//   set_frame_refs, motion field       decoder/Parser.cpp:584-911
//   skip mode, global motion           decoder/Parser.cpp:922-1125
//   Parser::parseTileGroup             decoder/Parser.cpp:474-524
//   motionVectorStorage, finishFrame   decoder/Parser.cpp:1699-1720, 1784-1818
// and the batch assembly of the oracle harness (oracle/harness/refdump.cpp fillHeader /
// fillFrameTables), which defines what the backend receives.
#include <stdarg.h>
#include <system_error>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <new>
#include <thread>

#include "parser.h"

namespace av1p {

void Cdfs::reset_counters()
{
    uint16_t* c = reinterpret_cast<uint16_t*>(&coef);
    for (uint16_t o : kCoefCounters) c[o] = 0;
    uint16_t* m = reinterpret_cast<uint16_t*>(&mode);
    for (uint16_t o : kModeCounters) m[o] = 0;
    for (auto& v : mv) {
        uint16_t* p = reinterpret_cast<uint16_t*>(&v);
        for (uint16_t o : kMvCounters) p[o] = 0;
        for (auto& comp : v.comp) {
            uint16_t* q = reinterpret_cast<uint16_t*>(&comp);
            for (uint16_t o : kMvCompCounters) q[o] = 0;
        }
    }
}

Parser::Parser() {}

int TileCtx::fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (err.empty()) err = buf;  // (the first failure of the tile)
    return code;
}

Parser::~Parser()
{
    for (TileCtx* t : par_tiles) delete t;
    for (Frame* f : spare) delete f;
}

Frame* Parser::take_frame()
{
    if (spare.empty()) return new Frame;
    Frame* f = spare.back();
    spare.pop_back();
    f->blocks.clear();
    f->mi.clear();
    f->tbs.clear();
    f->coefs.clear();
    f->palette.clear();
    f->cdef.clear();
    f->lr.clear();
    memset(&f->batch, 0, sizeof(f->batch));
    return f;
}

int Parser::fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    err = buf;
    return code;
}

#define CHK(x)                    \
    do {                          \
        int rc_ = (x);            \
        if (rc_) return rc_;      \
    } while (0)

// ------------------------------------------------------------------------------------
// sequence header (spec 5.5; Parser.cpp:288-436)
// ------------------------------------------------------------------------------------
int Parser::parse_sequence_header(BitReader& br)
{
    SeqHdr s;
    s.profile = br.f(3);
    s.still_picture = br.flag();
    s.reduced_still_picture_header = br.flag();
    if (s.reduced_still_picture_header) {
        s.operating_points = 1;
        s.op_idc[0] = 0;
        br.f(5);  // seq_level_idx[0]
    } else {
        s.timing_info_present = br.flag();
        if (s.timing_info_present) {
            br.f(32);  // num_units_in_display_tick
            br.f(32);  // time_scale
            s.equal_picture_interval = br.flag();
            if (s.equal_picture_interval) br.uvlc();
            s.decoder_model_info_present = br.flag();
            if (s.decoder_model_info_present) {
                s.buffer_delay_length = br.f(5) + 1;
                br.f(32);  // num_units_in_decoding_tick
                s.buffer_removal_time_length = br.f(5) + 1;
                s.frame_presentation_time_length = br.f(5) + 1;
            }
        }
        const bool initial_display_delay_present = br.flag();
        s.operating_points = br.f(5) + 1;
        for (int i = 0; i < s.operating_points; i++) {
            s.op_idc[i] = br.f(12);
            const int level = br.f(5);
            if (level > 7) br.f(1);  // seq_tier
            if (s.decoder_model_info_present) {
                s.decoder_model_present_for_op[i] = br.flag();
                if (s.decoder_model_present_for_op[i]) {
                    br.f(s.buffer_delay_length);  // decoder_buffer_delay
                    br.f(s.buffer_delay_length);  // encoder_buffer_delay
                    br.f(1);                      // low_delay_mode_flag
                }
            }
            if (initial_display_delay_present)
                if (br.flag()) br.f(4);
        }
    }
    s.frame_width_bits = br.f(4) + 1;
    s.frame_height_bits = br.f(4) + 1;
    s.max_frame_width = br.f(s.frame_width_bits) + 1;
    s.max_frame_height = br.f(s.frame_height_bits) + 1;
    s.frame_id_numbers_present = s.reduced_still_picture_header ? false : br.flag();
    if (s.frame_id_numbers_present) {
        s.delta_frame_id_length = br.f(4) + 2;
        s.additional_frame_id_length = br.f(3) + 1;
    }
    s.use_128x128 = br.flag();
    s.enable_filter_intra = br.flag();
    s.enable_intra_edge_filter = br.flag();
    if (s.reduced_still_picture_header) {
        s.seq_force_screen_content_tools = 2;
        s.seq_force_integer_mv = 2;
    } else {
        s.enable_interintra_compound = br.flag();
        s.enable_masked_compound = br.flag();
        s.enable_warped_motion = br.flag();
        s.enable_dual_filter = br.flag();
        s.enable_order_hint = br.flag();
        if (s.enable_order_hint) {
            s.enable_jnt_comp = br.flag();
            s.enable_ref_frame_mvs = br.flag();
        }
        s.seq_force_screen_content_tools = br.flag() ? 2 : (int)br.f(1);
        if (s.seq_force_screen_content_tools > 0) s.seq_force_integer_mv = br.flag() ? 2 : (int)br.f(1);
        else s.seq_force_integer_mv = 2;
        if (s.enable_order_hint) s.order_hint_bits = br.f(3) + 1;
    }
    s.enable_superres = br.flag();
    s.enable_cdef = br.flag();
    s.enable_restoration = br.flag();
    // color_config (Parser.cpp:197-270)
    const bool high_bitdepth = br.flag();
    if (s.profile == 2 && high_bitdepth) s.bit_depth = br.flag() ? 12 : 10;
    else if (s.profile <= 2) s.bit_depth = high_bitdepth ? 10 : 8;
    else return fail(AV1R_E_UNSUPPORTED, "seq_profile %d", s.profile);
    s.mono_chrome = s.profile == 1 ? false : br.flag();
    s.num_planes = s.mono_chrome ? 1 : 3;
    int cp = 2, tc = 2, mc = 2;
    if (br.flag()) {
        cp = br.f(8);
        tc = br.f(8);
        mc = br.f(8);
    }
    if (s.mono_chrome) {
        br.f(1);  // color_range
        s.subx = s.suby = true;
    } else if (cp == 1 && tc == 13 && mc == 0) {  // BT709 / SRGB / IDENTITY
        s.subx = s.suby = false;
    } else {
        br.f(1);  // color_range
        if (s.profile == 0) {
            s.subx = s.suby = true;
        } else if (s.profile == 1) {
            s.subx = s.suby = false;
        } else if (s.bit_depth == 12) {
            s.subx = br.flag();
            s.suby = s.subx ? br.flag() : false;
        } else {
            s.subx = true;
            s.suby = false;
        }
        if (s.subx && s.suby) br.f(2);  // chroma_sample_position
    }
    if (!s.mono_chrome) s.separate_uv_delta_q = br.flag();
    s.film_grain_params_present = br.flag();
    if (br.over) return fail(AV1R_E_INVALID, "truncated sequence header");
    // the reference's support (README: 8-bit 4:2:0 only)
    if (s.bit_depth != 8 || !s.subx || !s.suby || s.mono_chrome)
        return fail(AV1R_E_UNSUPPORTED, "only 8-bit 4:2:0 streams are supported");
    seq = s;
    have_seq = true;
    return AV1R_OK;
}

// ------------------------------------------------------------------------------------
// frame header helpers
// ------------------------------------------------------------------------------------
int Parser::relative_dist(int a, int b) const  // get_relative_dist (Parser.cpp:712-721)
{
    if (!seq.enable_order_hint) return 0;
    int diff = a - b;
    const int m = 1 << (seq.order_hint_bits - 1);
    diff = (diff & (m - 1)) - (diff & m);
    return diff;
}

void Parser::compute_image_size()
{
    fh.mi_cols = 2 * ((fh.frame_width + 7) >> 3);
    fh.mi_rows = 2 * ((fh.frame_height + 7) >> 3);
    const int align = seq.use_128x128 ? 128 : 64;  // computeAlignedSize (Parser.cpp:1424-1429)
    fh.aligned_mi_cols = ((fh.frame_width + align - 1) & ~(align - 1)) >> 2;
    fh.aligned_mi_rows = ((fh.frame_height + align - 1) & ~(align - 1)) >> 2;
}

int Parser::superres_params(BitReader& br)
{
    fh.use_superres = seq.enable_superres ? br.flag() : false;
    fh.superres_denom = fh.use_superres ? (int)br.f(3) + 9 : 8;
    fh.upscaled_width = fh.frame_width;
    fh.frame_width = (fh.upscaled_width * 8 + fh.superres_denom / 2) / fh.superres_denom;
    if (fh.use_superres) return fail(AV1R_E_UNSUPPORTED, "superres (the reference asserts, Av1Decoder.cpp:194-201)");
    return AV1R_OK;
}

int Parser::frame_size(BitReader& br)
{
    if (fh.frame_size_override) {
        fh.frame_width = br.f(seq.frame_width_bits) + 1;
        fh.frame_height = br.f(seq.frame_height_bits) + 1;
    } else {
        fh.frame_width = seq.max_frame_width;
        fh.frame_height = seq.max_frame_height;
    }
    CHK(superres_params(br));
    compute_image_size();
    return AV1R_OK;
}

int Parser::render_size(BitReader& br)
{
    if (br.flag()) {
        fh.render_width = br.f(16) + 1;
        fh.render_height = br.f(16) + 1;
    } else {
        fh.render_width = fh.upscaled_width;
        fh.render_height = fh.frame_height;
    }
    return AV1R_OK;
}

int Parser::frame_size_with_refs(BitReader& br)
{
    bool found = false;
    for (int i = 0; i < kRefsPerFrame && !found; i++) {
        found = br.flag();
        if (found) {
            const RefSlot& r = slots[fh.ref_frame_idx[i]];
            fh.upscaled_width = r.upscaled_width;
            fh.frame_width = fh.upscaled_width;
            fh.frame_height = r.frame_height;
            fh.render_width = r.render_width;
            fh.render_height = r.render_height;
        }
    }
    if (!found) {
        CHK(frame_size(br));
        CHK(render_size(br));
    } else {
        CHK(superres_params(br));
        compute_image_size();
    }
    return AV1R_OK;
}

// set_frame_refs (spec 7.8; SetFrameRefs, Parser.cpp:584-710)
void Parser::set_frame_refs(int last_idx, int gold_idx)
{
    int* idx = fh.ref_frame_idx;
    for (int i = 0; i < kRefsPerFrame; i++) idx[i] = -1;
    idx[LAST_FRAME - LAST_FRAME] = last_idx;
    idx[GOLDEN_FRAME - LAST_FRAME] = gold_idx;
    bool used[8] = {};
    used[last_idx] = used[gold_idx] = true;
    const int curHint = 1 << (seq.order_hint_bits - 1);
    int shifted[8];
    for (int i = 0; i < 8; i++) shifted[i] = curHint + relative_dist(slots[i].order_hint, fh.order_hint);
    auto latest_backward = [&]() {
        int ref = -1, best = 0;
        for (int i = 0; i < 8; i++)
            if (!used[i] && shifted[i] >= curHint && (ref < 0 || shifted[i] >= best)) ref = i, best = shifted[i];
        return ref;
    };
    auto earliest_backward = [&]() {
        int ref = -1, best = 0;
        for (int i = 0; i < 8; i++)
            if (!used[i] && shifted[i] >= curHint && (ref < 0 || shifted[i] < best)) ref = i, best = shifted[i];
        return ref;
    };
    auto latest_forward = [&]() {
        int ref = -1, best = 0;
        for (int i = 0; i < 8; i++)
            if (!used[i] && shifted[i] < curHint && (ref < 0 || shifted[i] >= best)) ref = i, best = shifted[i];
        return ref;
    };
    auto set = [&](int refFrame, int r) {
        if (r >= 0) {
            idx[refFrame - LAST_FRAME] = r;
            used[r] = true;
        }
    };
    set(ALTREF_FRAME, latest_backward());
    set(BWDREF_FRAME, earliest_backward());
    set(ALTREF2_FRAME, earliest_backward());
    static const int order[5] = {LAST2_FRAME, LAST3_FRAME, BWDREF_FRAME, ALTREF2_FRAME, ALTREF_FRAME};
    for (int rf : order)
        if (idx[rf - LAST_FRAME] < 0) set(rf, latest_forward());
    int ref = -1, earliest = 0;
    for (int i = 0; i < 8; i++)
        if (ref < 0 || shifted[i] < earliest) ref = i, earliest = shifted[i];
    for (int i = 0; i < kRefsPerFrame; i++)
        if (idx[i] < 0) idx[i] = ref;
}

// tile_info (spec 5.9.15; Parser.cpp:1563-1643)
int Parser::tile_info(BitReader& br)
{
    auto tile_log2 = [](int blk, int target) {
        int k = 0;
        while ((blk << k) < target) k++;
        return k;
    };
    const int sbCols = seq.use_128x128 ? (fh.mi_cols + 31) >> 5 : (fh.mi_cols + 15) >> 4;
    const int sbRows = seq.use_128x128 ? (fh.mi_rows + 31) >> 5 : (fh.mi_rows + 15) >> 4;
    const int sbShift = seq.use_128x128 ? 5 : 4;
    const int sbSize = sbShift + 2;
    const int maxTileWidthSb = 4096 >> sbSize;
    int maxTileAreaSb = (4096 * 2304) >> (2 * sbSize);
    const int minLog2TileCols = tile_log2(maxTileWidthSb, sbCols);
    const int maxLog2TileCols = tile_log2(1, std::min(sbCols, 64));
    const int maxLog2TileRows = tile_log2(1, std::min(sbRows, 64));
    const int minLog2Tiles = std::max(minLog2TileCols, tile_log2(maxTileAreaSb, sbRows * sbCols));
    fh.mi_col_starts.clear();
    fh.mi_row_starts.clear();
    if (br.flag()) {  // uniform_tile_spacing_flag
        fh.tile_cols_log2 = minLog2TileCols;
        while (fh.tile_cols_log2 < maxLog2TileCols && br.flag()) fh.tile_cols_log2++;
        const int tileWidthSb = (sbCols + (1 << fh.tile_cols_log2) - 1) >> fh.tile_cols_log2;
        for (int start = 0; start < sbCols; start += tileWidthSb) fh.mi_col_starts.push_back(start << sbShift);
        fh.mi_col_starts.push_back(fh.mi_cols);
        const int minLog2TileRows = std::max(minLog2Tiles - fh.tile_cols_log2, 0);
        fh.tile_rows_log2 = minLog2TileRows;
        while (fh.tile_rows_log2 < maxLog2TileRows && br.flag()) fh.tile_rows_log2++;
        const int tileHeightSb = (sbRows + (1 << fh.tile_rows_log2) - 1) >> fh.tile_rows_log2;
        for (int start = 0; start < sbRows; start += tileHeightSb) fh.mi_row_starts.push_back(start << sbShift);
        fh.mi_row_starts.push_back(fh.mi_rows);
    } else {
        int widest = 0, start = 0;
        while (start < sbCols && fh.mi_col_starts.size() < 64) {
            fh.mi_col_starts.push_back(start << sbShift);
            const int maxWidth = std::min(sbCols - start, maxTileWidthSb);
            const int size = (int)br.ns(maxWidth) + 1;
            widest = std::max(widest, size);
            start += size;
        }
        fh.mi_col_starts.push_back(fh.mi_cols);
        fh.tile_cols_log2 = tile_log2(1, (int)fh.mi_col_starts.size() - 1);
        maxTileAreaSb = minLog2Tiles > 0 ? (sbRows * sbCols) >> (minLog2Tiles + 1) : sbRows * sbCols;
        const int maxTileHeightSb = std::max(maxTileAreaSb / std::max(widest, 1), 1);
        start = 0;
        while (start < sbRows && fh.mi_row_starts.size() < 64) {
            fh.mi_row_starts.push_back(start << sbShift);
            const int maxHeight = std::min(sbRows - start, maxTileHeightSb);
            start += (int)br.ns(maxHeight) + 1;
        }
        fh.mi_row_starts.push_back(fh.mi_rows);
        fh.tile_rows_log2 = tile_log2(1, (int)fh.mi_row_starts.size() - 1);
    }
    fh.tile_cols = (int)fh.mi_col_starts.size() - 1;
    fh.tile_rows = (int)fh.mi_row_starts.size() - 1;
    if (fh.tile_cols_log2 > 0 || fh.tile_rows_log2 > 0) {
        fh.context_update_tile_id = br.f(fh.tile_rows_log2 + fh.tile_cols_log2);
        fh.tile_size_bytes = br.f(2) + 1;
    } else {
        fh.context_update_tile_id = 0;
    }
    return AV1R_OK;
}

int Parser::read_delta_q(BitReader& br) { return br.flag() ? br.su(7) : 0; }

// decode_signed_subexp_with_ref and friends over the header bit reader (spec 5.9.26-28)
static int inverse_recenter(int r, int v)
{
    if (v > 2 * r) return v;
    if (v & 1) return r - ((v + 1) >> 1);
    return r + (v >> 1);
}
static int decode_subexp(BitReader& br, int numSyms)
{
    int i = 0, mk = 0;
    const int k = 3;
    for (;;) {
        const int b2 = i ? k + i - 1 : k;
        const int a = 1 << b2;
        if (numSyms <= mk + 3 * a) return (int)br.ns(numSyms - mk) + mk;
        if (br.flag()) {
            i++;
            mk += a;
        } else {
            return (int)br.f(b2) + mk;
        }
    }
}
static int decode_signed_subexp_with_ref(BitReader& br, int low, int high, int r)
{
    const int mx = high - low;
    r -= low;
    const int v = decode_subexp(br, mx);
    const int x = (r << 1) <= mx ? inverse_recenter(r, v) : mx - 1 - inverse_recenter(mx - 1 - r, v);
    return x + low;
}

// global_motion_params (spec 5.9.24; Parser.cpp:1045-1125)
int Parser::global_motion_params(BitReader& br)
{
    for (int ref = LAST_FRAME; ref <= ALTREF_FRAME; ref++) {
        fh.gm_type[ref] = AV1R_GM_IDENTITY;
        for (int i = 0; i < 6; i++) fh.gm_params[ref][i] = (i % 3 == 2) ? 1 << kWarpPrecBits : 0;
    }
    if (fh.frame_is_intra) return AV1R_OK;
    for (int ref = LAST_FRAME; ref <= ALTREF_FRAME; ref++) {
        int type = AV1R_GM_IDENTITY;
        if (br.flag()) {
            if (br.flag()) type = AV1R_GM_ROTZOOM;
            else type = br.flag() ? AV1R_GM_TRANSLATION : AV1R_GM_AFFINE;
        }
        fh.gm_type[ref] = type;
        auto param = [&](int idx) {
            int absBits = 12, precBits = 15;
            if (idx < 2) {
                if (type == AV1R_GM_TRANSLATION) {
                    absBits = 9 - !fh.allow_high_precision_mv;
                    precBits = 3 - !fh.allow_high_precision_mv;
                } else {
                    absBits = 12;
                    precBits = 6;
                }
            }
            const int precDiff = kWarpPrecBits - precBits;
            const int round = (idx % 3) == 2 ? (1 << kWarpPrecBits) : 0;
            const int sub = (idx % 3) == 2 ? (1 << precBits) : 0;
            const int mx = 1 << absBits;
            const int r = (fh.prev_gm[ref][idx] >> precDiff) - sub;
            fh.gm_params[ref][idx] = decode_signed_subexp_with_ref(br, -mx, mx + 1, r) * (1 << precDiff) + round;
        };
        if (type >= AV1R_GM_ROTZOOM) {
            param(2);
            param(3);
            if (type == AV1R_GM_AFFINE) {
                param(4);
                param(5);
            } else {
                fh.gm_params[ref][4] = -fh.gm_params[ref][3];
                fh.gm_params[ref][5] = fh.gm_params[ref][2];
            }
        }
        if (type >= AV1R_GM_TRANSLATION) {
            param(0);
            param(1);
        }
    }
    return AV1R_OK;
}

// film_grain_params (spec 5.9.30): read and discarded -- the reference synthesises no grain
// (it never parses these bits either; no conformance stream of bits/ carries grain)
int Parser::film_grain_params(BitReader& br)
{
    if (!seq.film_grain_params_present || (!fh.show_frame && !fh.showable_frame)) return AV1R_OK;
    if (!br.flag()) return AV1R_OK;  // apply_grain
    br.f(16);                        // grain_seed
    const bool update_grain = fh.frame_type == INTER_FRAME ? br.flag() : true;
    if (!update_grain) {
        br.f(3);  // film_grain_params_ref_idx
        return AV1R_OK;
    }
    const int numY = br.f(4);
    for (int i = 0; i < numY; i++) br.f(16);
    const bool chroma_from_luma = br.flag();
    int numCb = 0, numCr = 0;
    if (!chroma_from_luma) {
        numCb = br.f(4);
        for (int i = 0; i < numCb; i++) br.f(16);
        numCr = br.f(4);
        for (int i = 0; i < numCr; i++) br.f(16);
    }
    br.f(2);  // grain_scaling_minus_8
    const int lag = br.f(2);
    const int numPosLuma = 2 * lag * (lag + 1);
    const int numPosChroma = numY ? numPosLuma + 1 : numPosLuma;
    if (numY) br.f(8 * numPosLuma);
    if (chroma_from_luma || numCb) br.f(8 * numPosChroma);
    if (chroma_from_luma || numCr) br.f(8 * numPosChroma);
    br.f(2);  // ar_coeff_shift_minus_6
    br.f(2);  // grain_scale_shift
    if (numCb) br.f(8 + 8 + 9);
    if (numCr) br.f(8 + 8 + 9);
    br.f(1);  // overlap_flag
    br.f(1);  // clip_to_restricted_range
    return AV1R_OK;
}

void Parser::setup_past_independence()  // spec 7.20 (Parser.cpp:572-582, 1903-1935)
{
    for (int ref = LAST_FRAME; ref <= ALTREF_FRAME; ref++)
        for (int i = 0; i < 6; i++) fh.prev_gm[ref][i] = (i % 3 == 2) ? 1 << kWarpPrecBits : 0;
    fh.lf_delta_enabled = true;
    static const int8_t def[8] = {1, 0, 0, 0, -1, 0, -1, -1};
    memcpy(fh.lf_ref_deltas, def, 8);
    fh.lf_mode_deltas[0] = fh.lf_mode_deltas[1] = 0;
}

void Parser::load_previous()  // spec 7.21 (Parser.cpp:1132-1139)
{
    const RefSlot& r = slots[fh.ref_frame_idx[fh.primary_ref_frame]];
    memcpy(fh.prev_gm, r.saved_gm, sizeof(fh.prev_gm));
    memcpy(fh.lf_ref_deltas, r.lf_ref_deltas, 8);
    memcpy(fh.lf_mode_deltas, r.lf_mode_deltas, 2);
}

// skip_mode_params (spec 5.9.22; Parser.cpp:922-983)
int Parser::skip_mode_params(BitReader& br)
{
    bool allowed = false;
    if (!fh.frame_is_intra && fh.reference_select && seq.enable_order_hint) {
        int fwd = -1, bwd = -1, fwdHint = 0, bwdHint = 0;
        for (int i = 0; i < kRefsPerFrame; i++) {
            const int h = slots[fh.ref_frame_idx[i]].order_hint;
            if (relative_dist(h, fh.order_hint) < 0) {
                if (fwd < 0 || relative_dist(h, fwdHint) > 0) fwd = i, fwdHint = h;
            } else if (relative_dist(h, fh.order_hint) > 0) {
                if (bwd < 0 || relative_dist(h, bwdHint) < 0) bwd = i, bwdHint = h;
            }
        }
        if (fwd < 0) {
            allowed = false;
        } else if (bwd >= 0) {
            allowed = true;
            fh.skip_mode_frame[0] = LAST_FRAME + std::min(fwd, bwd);
            fh.skip_mode_frame[1] = LAST_FRAME + std::max(fwd, bwd);
        } else {
            int fwd2 = -1, fwd2Hint = 0;
            for (int i = 0; i < kRefsPerFrame; i++) {
                const int h = slots[fh.ref_frame_idx[i]].order_hint;
                if (relative_dist(h, fwdHint) < 0)
                    if (fwd2 < 0 || relative_dist(h, fwd2Hint) > 0) fwd2 = i, fwd2Hint = h;
            }
            if (fwd2 >= 0) {
                allowed = true;
                fh.skip_mode_frame[0] = LAST_FRAME + std::min(fwd, fwd2);
                fh.skip_mode_frame[1] = LAST_FRAME + std::max(fwd, fwd2);
            }
        }
    }
    fh.skip_mode_present = allowed ? br.flag() : false;
    return AV1R_OK;
}

// ------------------------------------------------------------------------------------
// motion field estimation (spec 7.9; Parser.cpp:772-910)
// ------------------------------------------------------------------------------------
static Mv mv_projection(Mv mv, int numerator, int denominator)
{
    static const int Div_Mult[32] = {0,    16384, 8192, 5461, 4096, 3276, 2730, 2340, 2048, 1820, 1638,
                                     1489, 1365,  1260, 1170, 1092, 1024, 963,  910,  862,  819,  780,
                                     744,  712,   682,  655,  630,  606,  585,  564,  546,  528};
    const int clippedDen = std::min(denominator, AV1R_MAX_FRAME_DISTANCE);
    const int clippedNum = std::max(-AV1R_MAX_FRAME_DISTANCE, std::min(AV1R_MAX_FRAME_DISTANCE, numerator));
    Mv out;
    const int v[2] = {mv.r, mv.c};
    int16_t o[2];
    for (int i = 0; i < 2; i++) {
        const int x = v[i] * clippedNum * Div_Mult[clippedDen];
        const int scaled = x >= 0 ? (x + (1 << 13)) >> 14 : -((-x + (1 << 13)) >> 14);
        o[i] = (int16_t)std::max(-(1 << 14) + 1, std::min((1 << 14) - 1, scaled));
    }
    out.r = o[0];
    out.c = o[1];
    return out;
}

bool Parser::mv_project(int src, int dstSign)
{
    const RefSlot& r = slots[fh.ref_frame_idx[src - LAST_FRAME]];
    if (r.mi_rows != fh.mi_rows || r.mi_cols != fh.mi_cols || r.frame_type == INTRA_ONLY_FRAME || r.frame_type == KEY_FRAME)
        return false;
    const int w8 = fh.mi_cols >> 1, h8 = fh.mi_rows >> 1;
    const int mfw = fh.aligned_mi_cols >> 1;
    auto project = [](int& v8, int delta, int sign, int max8, int maxOff8) {
        const int base8 = (v8 >> 3) << 3;
        const int off8 = delta >= 0 ? delta >> (3 + 1 + 2) : -((-delta) >> (3 + 1 + 2));
        v8 += sign * off8;
        return !(v8 < 0 || v8 >= max8 || v8 < base8 - maxOff8 || v8 >= base8 + 8 + maxOff8);
    };
    // the order-hint distances, once per call rather than per unit
    const int refToCur = relative_dist(fh.order_hints[src], fh.order_hint);
    int refOffsetOf[8], refToDst[8];
    for (int k = 0; k < 8; k++) refOffsetOf[k] = relative_dist(fh.order_hints[src], r.saved_order_hints[k]);
    for (int dst = LAST_FRAME; dst <= ALTREF_FRAME; dst++) refToDst[dst] = relative_dist(fh.order_hint, fh.order_hints[dst]);
    Mv* mf[8];
    for (int dst = LAST_FRAME; dst <= ALTREF_FRAME; dst++) mf[dst] = motion_field[dst].data();
    for (int y8 = 0; y8 < h8; y8++)
        for (int x8 = 0; x8 < w8; x8++) {
            const int srcRef = r.mf_ref[(size_t)y8 * w8 + x8];  // (unit 2 y8 + 1, 2 x8 + 1: motion vector storage)
            if (srcRef <= INTRA_FRAME) continue;
            const int refOffset = refOffsetOf[srcRef];
            if (!(abs(refToCur) <= AV1R_MAX_FRAME_DISTANCE && abs(refOffset) <= AV1R_MAX_FRAME_DISTANCE && refOffset > 0))
                continue;
            const Mv mv = r.mf_mv[(size_t)y8 * w8 + x8];
            Mv proj = mv_projection(mv, refToCur * dstSign, refOffset);
            int px = x8, py = y8;
            if (!(project(px, proj.c, dstSign, w8, 8) && project(py, proj.r, dstSign, h8, 0))) continue;
            for (int dst = LAST_FRAME; dst <= ALTREF_FRAME; dst++)
                mf[dst][(size_t)py * mfw + px] = mv_projection(mv, refToDst[dst], refOffset);
        }
    return true;
}

void Parser::motion_field_estimation()
{
    const size_t n = (size_t)(fh.aligned_mi_rows >> 1) * (fh.aligned_mi_cols >> 1);
    Mv invalid;
    invalid.r = invalid.c = (int16_t)INT16_MIN;
    for (int ref = LAST_FRAME; ref <= ALTREF_FRAME; ref++) motion_field[ref].assign(n, invalid);
    const int lastIdx = fh.ref_frame_idx[0];
    const int curGoldHint = fh.order_hints[GOLDEN_FRAME];
    const int lastAltHint = slots[lastIdx].saved_order_hints[ALTREF_FRAME];
    if (lastAltHint != curGoldHint) mv_project(LAST_FRAME, -1);
    int refStamp = 3 - 2;  // MFMV_STACK_SIZE - 2
    static const int srcs[3] = {BWDREF_FRAME, ALTREF2_FRAME, ALTREF_FRAME};
    for (int src : srcs) {
        bool use = relative_dist(fh.order_hints[src], fh.order_hint) > 0;
        if (src == ALTREF_FRAME && use) use = refStamp >= 0;
        if (use && mv_project(src, 1)) refStamp--;
    }
    if (refStamp >= 0) mv_project(LAST2_FRAME, -1);
}

// ------------------------------------------------------------------------------------
// uncompressed_header (spec 5.9.2; Parser.cpp:1152-1403)
// ------------------------------------------------------------------------------------
int Parser::parse_uncompressed_header(BitReader& br)
{
    const int allFrames = 0xff;
    fh = FrameHdr();
    int idLen = 0;
    if (seq.frame_id_numbers_present) idLen = seq.additional_frame_id_length + seq.delta_frame_id_length + 1;
    if (seq.reduced_still_picture_header) {
        fh.frame_type = KEY_FRAME;
        fh.frame_is_intra = true;
        fh.show_frame = true;
    } else {
        fh.show_existing_frame = br.flag();
        if (fh.show_existing_frame) {
            fh.frame_to_show = br.f(3);
            if (seq.decoder_model_info_present && !seq.equal_picture_interval) br.f(seq.frame_presentation_time_length);
            if (seq.frame_id_numbers_present) br.f(idLen);
            fh.frame_type = slots[fh.frame_to_show].frame_type;
            fh.refresh_frame_flags = fh.frame_type == KEY_FRAME ? allFrames : 0;
            if (!slots[fh.frame_to_show].valid) return fail(AV1R_E_INVALID, "show_existing_frame of an empty slot");
            return AV1R_OK;
        }
        fh.frame_type = br.f(2);
        fh.frame_is_intra = fh.frame_type == INTRA_ONLY_FRAME || fh.frame_type == KEY_FRAME;
        fh.show_frame = br.flag();
        if (fh.show_frame && seq.decoder_model_info_present && !seq.equal_picture_interval)
            br.f(seq.frame_presentation_time_length);
        fh.showable_frame = fh.show_frame ? fh.frame_type != KEY_FRAME : br.flag();
        fh.error_resilient = (fh.frame_type == SWITCH_FRAME || (fh.frame_type == KEY_FRAME && fh.show_frame)) ? true : br.flag();
    }
    if (fh.frame_type == KEY_FRAME && fh.show_frame) {
        for (auto& s : slots) {
            s.valid = false;
            s.order_hint = 0;
        }
        for (int i = 0; i < kRefsPerFrame; i++) fh.order_hints[LAST_FRAME + i] = 0;
    }
    fh.disable_cdf_update = br.flag();
    fh.allow_screen_content_tools = seq.seq_force_screen_content_tools == 2 ? br.flag() : seq.seq_force_screen_content_tools;
    if (fh.allow_screen_content_tools) fh.force_integer_mv = seq.seq_force_integer_mv == 2 ? br.flag() : seq.seq_force_integer_mv;
    if (fh.frame_is_intra) fh.force_integer_mv = true;
    if (seq.frame_id_numbers_present) {
        fh.current_frame_id = br.f(idLen);
        // mark_ref_frames (spec 7.5): frames too old to be referenced
        const int diffLen = seq.delta_frame_id_length;
        for (auto& s : slots) {
            if (!s.valid) continue;
            if (fh.current_frame_id > (1 << diffLen)) {
                if (s.frame_id > fh.current_frame_id || s.frame_id < fh.current_frame_id - (1 << diffLen)) s.valid = false;
            } else if (s.frame_id > fh.current_frame_id &&
                       s.frame_id < (1 << idLen) + fh.current_frame_id - (1 << diffLen)) {
                s.valid = false;
            }
        }
    }
    fh.frame_size_override = fh.frame_type == SWITCH_FRAME ? true : seq.reduced_still_picture_header ? false : br.flag();
    fh.order_hint = br.f(seq.order_hint_bits);
    fh.primary_ref_frame = (fh.frame_is_intra || fh.error_resilient) ? kPrimaryRefNone : (int)br.f(3);
    if (seq.decoder_model_info_present) {
        if (br.flag())  // buffer_removal_time_present_flag
            for (int op = 0; op < seq.operating_points; op++)
                if (seq.decoder_model_present_for_op[op]) {
                    const int idc = seq.op_idc[op];
                    // temporal / spatial id of this OBU are 0 (no extension support needed:
                    // idc 0 or layer 0 present)
                    if (idc == 0 || ((idc & 1) && (idc & 0x100))) br.f(seq.buffer_removal_time_length);
                }
    }
    fh.refresh_frame_flags = (fh.frame_type == SWITCH_FRAME || (fh.frame_type == KEY_FRAME && fh.show_frame)) ? allFrames : br.f(8);
    if ((!fh.frame_is_intra || fh.refresh_frame_flags != allFrames) && fh.error_resilient && seq.enable_order_hint)
        for (int i = 0; i < 8; i++) {
            const int hint = br.f(seq.order_hint_bits);
            if (hint != slots[i].order_hint) {
                slots[i].valid = false;
                slots[i].order_hint = hint;
            }
        }
    if (fh.frame_is_intra) {
        CHK(frame_size(br));
        CHK(render_size(br));
        if (fh.allow_screen_content_tools && fh.upscaled_width == fh.frame_width) fh.allow_intrabc = br.flag();
    } else {
        bool shortSignaling = false;
        if (seq.enable_order_hint) {
            shortSignaling = br.flag();
            if (shortSignaling) {
                const int last = br.f(3), gold = br.f(3);
                set_frame_refs(last, gold);
            }
        }
        for (int i = 0; i < kRefsPerFrame; i++) {
            if (!shortSignaling) fh.ref_frame_idx[i] = br.f(3);
            if (seq.frame_id_numbers_present) br.f(seq.delta_frame_id_length);
            if (!slots[fh.ref_frame_idx[i]].valid) return fail(AV1R_E_INVALID, "reference %d is an empty slot", i + 1);
        }
        if (fh.frame_size_override && !fh.error_resilient) {
            CHK(frame_size_with_refs(br));
        } else {
            CHK(frame_size(br));
            CHK(render_size(br));
        }
        fh.allow_high_precision_mv = fh.force_integer_mv ? false : br.flag();
        fh.interpolation_filter = br.flag() ? SWITCHABLE : (int)br.f(2);
        fh.is_motion_mode_switchable = br.flag();
        fh.use_ref_frame_mvs = (fh.error_resilient || !seq.enable_ref_frame_mvs) ? false : br.flag();
        for (int i = 0; i < kRefsPerFrame; i++) {
            const int refFrame = LAST_FRAME + i;
            const int hint = slots[fh.ref_frame_idx[i]].order_hint;
            fh.order_hints[refFrame] = hint;
            fh.ref_frame_sign_bias[refFrame] = seq.enable_order_hint ? relative_dist(hint, fh.order_hint) > 0 : false;
        }
    }
    fh.disable_frame_end_update_cdf = (seq.reduced_still_picture_header || fh.disable_cdf_update) ? true : br.flag();
    if (fh.primary_ref_frame == kPrimaryRefNone) {
        cdf.mode = kDefaultModeCdfs;
        cdf.mv[0] = kDefaultMvCdfs[0];
        cdf.mv[1] = kDefaultMvCdfs[1];
        setup_past_independence();
    } else {
        const RefSlot& r = slots[fh.ref_frame_idx[fh.primary_ref_frame]];
        cdf = r.cdfs;
        cdf.reset_counters();
        load_previous();
    }
    if (fh.use_ref_frame_mvs) motion_field_estimation();
    CHK(tile_info(br));
    // quantization_params (Parser.cpp:1733-1760)
    fh.base_q_idx = br.f(8);
    fh.delta_q_y_dc = read_delta_q(br);
    {
        const bool diff_uv_delta = seq.separate_uv_delta_q ? br.flag() : false;
        fh.delta_q_u_dc = read_delta_q(br);
        fh.delta_q_u_ac = read_delta_q(br);
        if (diff_uv_delta) {
            fh.delta_q_v_dc = read_delta_q(br);
            fh.delta_q_v_ac = read_delta_q(br);
        } else {
            fh.delta_q_v_dc = fh.delta_q_u_dc;
            fh.delta_q_v_ac = fh.delta_q_u_ac;
        }
    }
    fh.using_qmatrix = br.flag();
    if (fh.using_qmatrix) {
        br.f(4);
        br.f(4);
        if (seq.separate_uv_delta_q) br.f(4);
        return fail(AV1R_E_UNSUPPORTED, "quantizer matrices (the reference asserts, TransformBlock.cpp:1743)");
    }
    // segmentation_params: not supported by the reference (Parser.cpp:1820-1841 asserts)
    fh.segmentation_enabled = br.flag();
    if (fh.segmentation_enabled) return fail(AV1R_E_UNSUPPORTED, "segmentation (the reference asserts, Block.cpp:507,599)");
    // delta_q_params / delta_lf_params (Parser.cpp:1874-1901)
    if (fh.base_q_idx > 0) fh.delta_q_present = br.flag();
    if (fh.delta_q_present) fh.delta_q_res = br.f(2);
    if (fh.delta_q_present) {
        if (!fh.allow_intrabc) fh.delta_lf_present = br.flag();
        if (fh.delta_lf_present) {
            fh.delta_lf_res = br.f(2);
            fh.delta_lf_multi = br.flag();
        }
    }
    if (fh.primary_ref_frame == kPrimaryRefNone) {
        const int q = fh.base_q_idx;
        cdf.coef = kDefaultCoefCdfs[q <= 20 ? 0 : q <= 60 ? 1 : q <= 120 ? 2 : 3];
    }
    fh.coded_lossless = fh.base_q_idx == 0 && fh.delta_q_y_dc == 0 && fh.delta_q_u_ac == 0 && fh.delta_q_u_dc == 0 &&
                        fh.delta_q_v_ac == 0 && fh.delta_q_v_dc == 0;
    fh.all_lossless = fh.coded_lossless && fh.frame_width == fh.upscaled_width;
    // loop_filter_params (Parser.cpp:1937-1975)
    if (fh.coded_lossless || fh.allow_intrabc) {
        fh.lf_level[0] = fh.lf_level[1] = 0;
        static const int8_t def[8] = {1, 0, 0, 0, -1, 0, -1, -1};
        memcpy(fh.lf_ref_deltas, def, 8);
        fh.lf_mode_deltas[0] = fh.lf_mode_deltas[1] = 0;
    } else {
        fh.lf_level[0] = br.f(6);
        fh.lf_level[1] = br.f(6);
        if (fh.lf_level[0] || fh.lf_level[1]) {
            fh.lf_level[2] = br.f(6);
            fh.lf_level[3] = br.f(6);
        }
        fh.lf_sharpness = br.f(3);
        fh.lf_delta_enabled = br.flag();
        if (fh.lf_delta_enabled && br.flag()) {
            for (int i = 0; i < 8; i++)
                if (br.flag()) fh.lf_ref_deltas[i] = (int8_t)br.su(7);
            for (int i = 0; i < 2; i++)
                if (br.flag()) fh.lf_mode_deltas[i] = (int8_t)br.su(7);
        }
    }
    // cdef_params (Parser.cpp:1977-2006)
    if (fh.coded_lossless || fh.allow_intrabc || !seq.enable_cdef) {
        fh.cdef_bits = 0;
        fh.cdef_damping = 3;
    } else {
        fh.cdef_damping = br.f(2) + 3;
        fh.cdef_bits = br.f(2);
        for (int i = 0; i < (1 << fh.cdef_bits); i++) {
            fh.cdef_y_pri[i] = br.f(4);
            fh.cdef_y_sec[i] = br.f(2);
            if (fh.cdef_y_sec[i] == 3) fh.cdef_y_sec[i]++;
            fh.cdef_uv_pri[i] = br.f(4);
            fh.cdef_uv_sec[i] = br.f(2);
            if (fh.cdef_uv_sec[i] == 3) fh.cdef_uv_sec[i]++;
        }
    }
    // lr_params (Parser.cpp:2034-2111)
    if (!(fh.all_lossless || fh.allow_intrabc || !seq.enable_restoration)) {
        static const int remap[4] = {AV1R_RESTORE_NONE, AV1R_RESTORE_SWITCHABLE, AV1R_RESTORE_WIENER, AV1R_RESTORE_SGRPROJ};
        bool chroma = false;
        for (int i = 0; i < 3; i++) {
            fh.lr_type[i] = remap[br.f(2)];
            if (fh.lr_type[i] != AV1R_RESTORE_NONE) {
                fh.uses_lr = true;
                chroma |= i > 0;
            }
        }
        if (fh.uses_lr) {
            int shift;
            if (seq.use_128x128) {
                shift = br.f(1) + 1;
            } else {
                shift = br.f(1);
                if (shift) shift += br.f(1);
            }
            fh.lr_unit_size[0] = 256 >> (2 - shift);
            const int uvShift = chroma ? (int)br.f(1) : 0;
            fh.lr_unit_size[1] = fh.lr_unit_size[2] = fh.lr_unit_size[0] >> uvShift;
        }
    }
    fh.tx_mode = fh.coded_lossless ? TX_MODE_ONLY_4X4 : br.flag() ? TX_MODE_SELECT : TX_MODE_LARGEST;
    fh.reference_select = fh.frame_is_intra ? false : br.flag();
    CHK(skip_mode_params(br));
    fh.allow_warped_motion = (fh.frame_is_intra || fh.error_resilient || !seq.enable_warped_motion) ? false : br.flag();
    fh.reduced_tx_set = br.flag();
    CHK(global_motion_params(br));
    CHK(film_grain_params(br));
    if (br.over) return fail(AV1R_E_INVALID, "truncated frame header");
    if (fh.frame_width & 1 || fh.frame_height & 1) return fail(AV1R_E_UNSUPPORTED, "odd frame size %dx%d", fh.frame_width, fh.frame_height);
    if (fh.frame_width > seq.max_frame_width || fh.frame_height > seq.max_frame_height ||
        (int64_t)fh.frame_width * fh.frame_height > (int64_t)8192 * 4352)
        return fail(AV1R_E_UNSUPPORTED, "frame size %dx%d (sequence maximum %dx%d, library limit 8192x4352 pixels)",
                    fh.frame_width, fh.frame_height, seq.max_frame_width, seq.max_frame_height);
    return AV1R_OK;
}

// ------------------------------------------------------------------------------------
// frame start / end, reference update
// ------------------------------------------------------------------------------------
void Parser::start_frame()
{
    mi_stride = fh.aligned_mi_cols;
    MiInfo z;
    memset(&z, 0, sizeof(z));
    z.pal_idx = ~0u;
    mi.assign((size_t)fh.aligned_mi_rows * mi_stride, z);
    if (emit_mi) {
        mi_lftx.assign(mi.size() * 3, 0);
        mi_dlf.assign(mi.size() * 4, 0);
    }
    cdef_rows = (fh.mi_rows + 15) / 16;
    cdef_cols = (fh.mi_cols + 15) / 16;
    cdef_idx.assign((size_t)cdef_rows * cdef_cols, -1);
    lr_units.clear();
    for (int p = 0; p < 3; p++) {
        lr_off[p] = (int)lr_units.size();
        if (!fh.uses_lr || fh.lr_type[p] == AV1R_RESTORE_NONE) continue;
        const int sub = p ? 1 : 0;
        const int us = fh.lr_unit_size[p];
        fh.lr_unit_rows[p] = std::max((((fh.frame_height + sub) >> sub) + (us >> 1)) / us, 1);
        fh.lr_unit_cols[p] = std::max((((fh.upscaled_width + sub) >> sub) + (us >> 1)) / us, 1);
        av1r_lr_unit u;
        memset(&u, 0, sizeof(u));
        lr_units.insert(lr_units.end(), (size_t)fh.lr_unit_rows[p] * fh.lr_unit_cols[p], u);
    }
    cur = take_frame();
    memset(&cur->hdr, 0, sizeof(cur->hdr));
    fill_header(cur->hdr);
}

void Parser::fill_header(av1r_frame_hdr& o) const  // refdump.cpp fillHeader / fillFrameTables
{
    o.version = AV1R_VERSION;
    o.frame_width = fh.frame_width;
    o.frame_height = fh.frame_height;
    o.mi_cols = fh.mi_cols;
    o.mi_rows = fh.mi_rows;
    o.mi_stride = fh.aligned_mi_cols;
    o.mi_rows_alloc = fh.aligned_mi_rows;
    o.sb128 = seq.use_128x128;
    o.subx = seq.subx;
    o.suby = seq.suby;
    o.bitdepth = (uint8_t)seq.bit_depth;
    o.show_frame = fh.show_frame;
    o.show_existing_frame = fh.show_existing_frame;
    o.frame_to_show = (uint8_t)fh.frame_to_show;
    o.refresh_frame_flags = (uint8_t)fh.refresh_frame_flags;
    o.frame_type = (uint8_t)fh.frame_type;
    o.enable_intra_edge_filter = seq.enable_intra_edge_filter;
    o.force_integer_mv = fh.force_integer_mv;
    o.allow_intrabc = fh.allow_intrabc;
    for (int i = 0; i < 8; i++) o.ref_frame_idx[i] = i < kRefsPerFrame ? (int8_t)fh.ref_frame_idx[i] : -1;
    for (int r = 0; r < 8; r++) {
        o.gm_type[r] = (uint8_t)fh.gm_type[r];
        for (int k = 0; k < 6; k++) o.gm_params[r][k] = fh.gm_params[r][k];
        if (r >= LAST_FRAME && !fh.frame_is_intra) {
            const int d = abs(relative_dist(fh.order_hints[r], fh.order_hint));
            o.ref_dist[r] = (uint8_t)std::min(d, AV1R_MAX_FRAME_DISTANCE);
        }
    }
    o.delta_q_y_dc = (int8_t)fh.delta_q_y_dc;
    o.delta_q_u_dc = (int8_t)fh.delta_q_u_dc;
    o.delta_q_u_ac = (int8_t)fh.delta_q_u_ac;
    o.delta_q_v_dc = (int8_t)fh.delta_q_v_dc;
    o.delta_q_v_ac = (int8_t)fh.delta_q_v_ac;
    for (int i = 0; i < 4; i++) o.lf_level[i] = (uint8_t)fh.lf_level[i];
    o.lf_sharpness = (uint8_t)fh.lf_sharpness;
    o.lf_delta_enabled = fh.lf_delta_enabled;
    o.delta_lf_multi = fh.delta_lf_multi;
    memcpy(o.lf_ref_deltas, fh.lf_ref_deltas, 8);
    memcpy(o.lf_mode_deltas, fh.lf_mode_deltas, 2);
    o.cdef_damping = (uint8_t)fh.cdef_damping;
    o.cdef_bits = (uint8_t)fh.cdef_bits;
    for (int i = 0; i < 8; i++) {
        o.cdef_y_pri[i] = (uint8_t)fh.cdef_y_pri[i];
        o.cdef_y_sec[i] = (uint8_t)fh.cdef_y_sec[i];
        o.cdef_uv_pri[i] = (uint8_t)fh.cdef_uv_pri[i];
        o.cdef_uv_sec[i] = (uint8_t)fh.cdef_uv_sec[i];
    }
    if (fh.show_existing_frame) return;
    o.cdef_rows = (fh.mi_rows + 15) / 16;
    o.cdef_cols = (fh.mi_cols + 15) / 16;
    o.uses_lr = fh.uses_lr;
    for (int p = 0; p < 3; p++) {
        o.lr_type[p] = (uint8_t)fh.lr_type[p];
        o.lr_unit_off[p] = lr_off[p];
        if (!fh.uses_lr || fh.lr_type[p] == AV1R_RESTORE_NONE) continue;
        o.lr_unit_size[p] = fh.lr_unit_size[p];
        o.lr_unit_rows[p] = fh.lr_unit_rows[p];
        o.lr_unit_cols[p] = fh.lr_unit_cols[p];
    }
}

// decode_frame_wrapup (spec 7.4 / Av1Decoder.cpp:141-153): the batch's frame tables,
// motion vector storage (7.19), the reference update (7.20)
int Parser::finish_frame()
{
    Frame& F = *cur;
    // CDFs of the context_update_tile_id tile (Tile::frame_end_update_cdf)
    if (!fh.disable_frame_end_update_cdf) cdf = saved_cdf;
    // mode-info grid (refdump.cpp fillFrameTables); left out when the consumer rebuilds
    // it on the device from the block records (av1p_set_mode_info(ctx, 0))
    F.mi.resize(emit_mi ? mi.size() : 0);  // (value-initialised: every field not set below is 0)
    for (size_t i = 0; i < F.mi.size(); i++) {
        const MiInfo& m = mi[i];
        av1r_mi& d = F.mi[i];
        for (int l = 0; l < 2; l++) {
            d.mv[l][0] = m.mv[l].r;
            d.mv[l][1] = m.mv[l].c;
            d.ref_frame[l] = m.ref[l];
        }
        d.mi_size = m.mi_size;
        d.y_mode = m.y_mode;
        d.uv_mode = m.uv_mode;
        d.filt = (uint8_t)((m.interp[0] & 15) | (m.interp[1] << 4));
        d.flags = (m.skip ? AV1R_MI_SKIP : 0) | (m.is_inter ? AV1R_MI_INTER : 0);
        for (int p = 0; p < 3; p++) d.lf_tx[p] = mi_lftx[i * 3 + p];
        for (int k = 0; k < 4; k++) d.delta_lf[k] = mi_dlf[i * 4 + k];
    }
    F.cdef = cdef_idx;
    F.lr = lr_units;
    // motion vector storage (Parser.cpp:1699-1720); which references lie behind this frame,
    // once per frame rather than per unit
    bool behind[8] = {};
    for (int r = INTRA_FRAME + 1; r < 8; r++) behind[r] = relative_dist(fh.order_hints[r], fh.order_hint) < 0;
    // Only the units the motion-field projection reads are stored: (2 y8 + 1, 2 x8 + 1) of every
    // 8x8 (the motion field projection, spec 7.9.2 / Parser.cpp:772-910, reads no other unit), a quarter of the grid,
    // which the reference slots then copy
    const int h8 = fh.mi_rows >> 1, w8 = fh.mi_cols >> 1;
    mf_ref.assign((size_t)h8 * w8, -1);
    mf_mv.assign((size_t)h8 * w8, Mv());
    for (int y8 = 0; y8 < h8; y8++)
        for (int x8 = 0; x8 < w8; x8++) {
            const MiInfo& m = mi_at(2 * y8 + 1, 2 * x8 + 1);
            for (int list = 0; list < 2; list++) {
                const int r = m.ref[list];
                if (r > INTRA_FRAME && behind[r]) {
                    const int lim = (1 << 12) - 1;
                    if (abs(m.mv[list].r) <= lim && abs(m.mv[list].c) <= lim) {
                        mf_ref[(size_t)y8 * w8 + x8] = (int8_t)r;
                        mf_mv[(size_t)y8 * w8 + x8] = m.mv[list];
                    }
                }
            }
        }
    reference_update();
    F.bind();
    done.push_back(cur);
    cur = nullptr;
    return AV1R_OK;
}

void Parser::reference_update()  // Parser::finishFrame (Parser.cpp:1784-1818)
{
    for (int i = 0; i < 8; i++) {
        if (!(fh.refresh_frame_flags & (1 << i))) continue;
        RefSlot& r = slots[i];
        r.valid = true;
        r.frame_id = fh.current_frame_id;
        r.upscaled_width = fh.upscaled_width;
        r.frame_width = fh.frame_width;
        r.frame_height = fh.frame_height;
        r.render_width = fh.render_width;
        r.render_height = fh.render_height;
        r.mi_cols = fh.mi_cols;
        r.mi_rows = fh.mi_rows;
        r.frame_type = fh.frame_type;
        r.order_hint = fh.order_hint;
        for (int j = 0; j < 8; j++) r.saved_order_hints[j] = fh.order_hints[j];
        r.mf_ref = mf_ref;
        r.mf_mv = mf_mv;
        r.cdfs = cdf;
        memcpy(r.saved_gm, fh.gm_params, sizeof(r.saved_gm));
        memcpy(r.lf_ref_deltas, fh.lf_ref_deltas, 8);
        memcpy(r.lf_mode_deltas, fh.lf_mode_deltas, 2);
        r.showable = fh.showable_frame;
    }
}

// show_existing_frame (spec 7.21 reference frame loading; Av1Decoder.cpp:158-169)
void Parser::show_existing()
{
    Frame* F = take_frame();
    memset(&F->hdr, 0, sizeof(F->hdr));
    const RefSlot& r = slots[fh.frame_to_show];
    // the header the harness records for it (refdump.cpp showExisting: fillHeader only)
    fh.frame_width = r.frame_width;
    fh.frame_height = r.frame_height;
    fill_header(F->hdr);
    F->hdr.frame_width = 0;
    F->hdr.frame_height = 0;
    F->hdr.mi_cols = F->hdr.mi_rows = F->hdr.mi_stride = F->hdr.mi_rows_alloc = 0;
    F->bind();
    done.push_back(F);
    if (fh.frame_type == KEY_FRAME) {
        // a shown key frame refreshes every slot with the shown one (spec 7.21)
        const RefSlot keep = r;
        fh.refresh_frame_flags = 0xff;
        for (int i = 0; i < 8; i++) slots[i] = keep;
    }
}

// ------------------------------------------------------------------------------------
// OBU loop (Decoder::decode, Av1Decoder.cpp:49-109)
// ------------------------------------------------------------------------------------
int Parser::parse_frame_header(BitReader& br)
{
    if (!have_seq) return fail(AV1R_E_INVALID, "frame header before any sequence header");
    if (seen_frame_header) return AV1R_OK;  // frame_header_copy
    CHK(parse_uncompressed_header(br));
    if (fh.show_existing_frame) {
        show_existing();
        seen_frame_header = false;
        return AV1R_OK;
    }
    tile_num = 0;
    seen_frame_header = true;
    start_frame();
    return AV1R_OK;
}

int Parser::decode_tu(const uint8_t* data, size_t size)
{
    done.clear();
    size_t pos = 0;
    while (pos < size) {
        BitReader hb(data + pos, size - pos);
        if (hb.f(1)) return fail(AV1R_E_INVALID, "obu_forbidden_bit");
        const int type = hb.f(4);
        const bool ext = hb.flag();
        const bool hasSize = hb.flag();
        hb.f(1);
        if (ext) hb.f(8);
        const uint64_t obuSize = hasSize ? hb.leb128() : (size - pos) - 1 - (ext ? 1 : 0);
        const size_t hdrBytes = hb.byte_pos();
        if (hb.over || pos + hdrBytes + obuSize > size) return fail(AV1R_E_INVALID, "truncated OBU");
        const uint8_t* payload = data + pos + hdrBytes;
        BitReader br(payload, (size_t)obuSize);
        int rc = AV1R_OK;
        switch (type) {
        case OBU_SEQUENCE_HEADER: rc = parse_sequence_header(br); break;
        case OBU_TEMPORAL_DELIMITER: seen_frame_header = false; break;
        case OBU_FRAME_HEADER:
        case OBU_REDUNDANT_FRAME_HEADER: rc = parse_frame_header(br); break;
        case OBU_FRAME:
            rc = parse_frame_header(br);
            if (!rc) {
                br.byte_align();
                rc = tile_group(br, payload, (size_t)obuSize);
            }
            break;
        case OBU_TILE_GROUP:
            if (!seen_frame_header) return fail(AV1R_E_INVALID, "tile group without a frame header");
            rc = tile_group(br, payload, (size_t)obuSize);
            break;
        default: break;  // metadata, tile list, padding
        }
        if (rc) return rc;
        pos += hdrBytes + (size_t)obuSize;
    }
    return AV1R_OK;
}

// tile_group_obu (spec 5.11.1; Parser::parseTileGroup, Parser.cpp:474-524)
int Parser::tile_group(BitReader& br, const uint8_t* data, size_t size)
{
    const int numTiles = fh.tile_cols * fh.tile_rows;
    const size_t start = br.pos;
    int tgStart = 0, tgEnd = numTiles - 1;
    if (numTiles > 1 && br.flag()) {
        const int bits = fh.tile_cols_log2 + fh.tile_rows_log2;
        tgStart = br.f(bits);
        tgEnd = br.f(bits);
    }
    br.byte_align();
    size_t off = br.byte_pos();
    (void)start;
    if (tgStart > tgEnd || tgEnd >= numTiles || tgStart != tile_num || !cur)
        return fail(AV1R_E_INVALID, "tile group %d..%d does not continue the frame (next tile %d of %d)", tgStart, tgEnd,
                    tile_num, numTiles);
    // the tiles' byte ranges (tile_size_minus_1 prefixes), then their parse
    struct TileSpan {
        size_t off, size;
    };
    std::vector<TileSpan> spans;
    for (int tn = tgStart; tn <= tgEnd; tn++) {
        size_t tileSize;
        if (tn == tgEnd) {
            tileSize = size - off;
        } else {
            if (off + fh.tile_size_bytes > size) return fail(AV1R_E_INVALID, "truncated tile size");
            uint32_t t = 0;
            for (int i = 0; i < fh.tile_size_bytes; i++) t |= (uint32_t)data[off + i] << (8 * i);
            off += fh.tile_size_bytes;
            tileSize = (size_t)t + 1;
        }
        if (off + tileSize > size) return fail(AV1R_E_INVALID, "tile %d size %zu exceeds the tile group", tn, tileSize);
        spans.push_back({off, tileSize});
        off += tileSize;
    }
    const int n = tgEnd - tgStart + 1;
    const int nThreads = std::min(tile_threads, n);
    if (nThreads <= 1) {
        for (int i = 0; i < n; i++) {
            begin_tile(tile, tgStart + i, data + spans[i].off, spans[i].size);
            const int rc = decode_tile(tile);
            CHK(merge_tile(tile, tgStart + i));
            if (rc) return rc;
            tile_num = tgStart + i + 1;
        }
    } else {
        // tile-parallel: every tile into its own context, the threads pulling tile indices
        while ((int)par_tiles.size() < n) par_tiles.push_back(new TileCtx);
        std::atomic<int> next{0};
        std::vector<int> rcs(n, AV1R_OK);
        auto work = [&]() {
            for (int i; (i = next.fetch_add(1)) < n;) {
                try {
                    begin_tile(*par_tiles[i], tgStart + i, data + spans[i].off, spans[i].size);
                    rcs[i] = decode_tile(*par_tiles[i]);
                } catch (const std::bad_alloc&) {
                    par_tiles[i]->err = "out of memory";
                    rcs[i] = AV1R_E_NOMEM;
                }
            }
        };
        // a thread that cannot be started (EAGAIN under a thread limit, or no memory for
        // its stack) is simply not there: the threads already running and this one share
        // the tiles through `next`, and every started thread is joined before leaving
        std::vector<std::thread> pool;
        pool.reserve(nThreads);
        for (int k = 1; k < nThreads; k++) {
            try {
                pool.emplace_back(work);
            } catch (const std::system_error&) {
                break;
            } catch (const std::bad_alloc&) {
                break;
            }
        }
        work();
        for (auto& th : pool) th.join();
        for (int i = 0; i < n; i++) {  // merged in tile order: the serial path's records
            CHK(merge_tile(*par_tiles[i], tgStart + i));
            if (rcs[i]) return rcs[i];
            tile_num = tgStart + i + 1;
        }
    }
    if (tgEnd == numTiles - 1) {
        CHK(finish_frame());
        seen_frame_header = false;
    }
    return AV1R_OK;
}

void Parser::begin_tile(TileCtx& T, int tn, const uint8_t* data, size_t size)
{
    const int tileRow = tn / fh.tile_cols, tileCol = tn % fh.tile_cols;
    T.mi_row_start = fh.mi_row_starts[tileRow];
    T.mi_row_end = fh.mi_row_starts[tileRow + 1];
    T.mi_col_start = fh.mi_col_starts[tileCol];
    T.mi_col_end = fh.mi_col_starts[tileCol + 1];
    T.current_q = fh.base_q_idx;
    T.tcdf = cdf;
    T.sd.init(data, size, fh.disable_cdf_update);
    T.pal_colors.clear();
    T.blocks.clear();
    T.tbs.clear();
    T.coefs.clear();
    T.palette.clear();
    T.err.clear();
}

int Parser::merge_tile(TileCtx& T, int tn)
{
    if (!T.err.empty()) err = T.err;
    if (tn == fh.context_update_tile_id) saved_cdf = T.tcdf;
    Frame& F = *cur;
    if (F.blocks.empty() && F.tbs.empty() && F.coefs.empty() && F.palette.empty()) {
        // the frame's first records: taken over as they are (indices already frame-relative)
        F.blocks.swap(T.blocks);
        F.tbs.swap(T.tbs);
        F.coefs.swap(T.coefs);
        F.palette.swap(T.palette);
        return AV1R_OK;
    }
    const uint32_t blk0 = (uint32_t)F.blocks.size(), tb0 = (uint32_t)F.tbs.size(), coef0 = (uint32_t)F.coefs.size(),
                   pal0 = (uint32_t)F.palette.size();
    for (av1r_block& b : T.blocks) {
        b.first_tb += tb0;
        if (b.palette_size_y || b.palette_size_uv) b.palette_off += pal0;
    }
    for (av1r_tb& t : T.tbs) {
        t.block += blk0;
        t.coef_off += coef0;
    }
    F.blocks.insert(F.blocks.end(), T.blocks.begin(), T.blocks.end());
    F.tbs.insert(F.tbs.end(), T.tbs.begin(), T.tbs.end());
    F.coefs.insert(F.coefs.end(), T.coefs.begin(), T.coefs.end());
    F.palette.insert(F.palette.end(), T.palette.begin(), T.palette.end());
    return AV1R_OK;
}

void Frame::bind()
{
    memset(&batch, 0, sizeof(batch));
    batch.hdr = &hdr;
    batch.mi = mi.empty() ? nullptr : mi.data();
    batch.blocks = blocks.data();
    batch.n_blocks = (uint32_t)blocks.size();
    batch.tbs = tbs.data();
    batch.n_tbs = (uint32_t)tbs.size();
    batch.coefs = coefs.data();
    batch.n_coefs = (uint32_t)coefs.size();
    batch.palette = palette.data();
    batch.n_palette = (uint32_t)palette.size();
    batch.cdef_idx = cdef.data();
    batch.lr_units = lr.data();
    batch.n_lr_units = (uint32_t)lr.size();
}

}  // namespace av1p
