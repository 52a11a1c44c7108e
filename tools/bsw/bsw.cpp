// bsw.cpp -- synthetic AV1 bitstream writer.
//
// Writes seeded 8-bit 4:2:0 AV1 streams (IVF) that any conformant decoder -- the reference
// CPU decoder included -- decodes, so the 1080p / 4K / multi-tile configurations of
// BASELINE.json get reference MD5s and a directly timed reference CPU rate, and the bench can
// decode real bitstreams end to end.
//
// How: the host parser's own syntax walk (av1dec_amd/csrc/parse, compiled here with
// -DAV1P_WRITER) runs in "write mode".  Every symbol it would read is instead chosen by this
// file's chooser and arithmetic-coded with the od_ec range encoder (the inverse of
// SymbolDecoder::read, AV1 spec 8.2.6), and the walk continues with the chosen value, so every
// context, CDF adaptation and derived quantity is exactly what a decoder will see.  Frame and
// sequence headers are written by hand for the feature set below and parsed back by the same
// parser (a header that does not parse to the bit count written is an error).  With verify on,
// each temporal unit is decoded again by an independent parser instance and its frame batches
// must equal the writer's own, field by field.
//
// The chooser samples each syntax element from the specification's default CDF for its
// context (a stable distribution: sampling from the adapted CDF would random-walk toward
// degenerate ones), with the overrides SURVEY.md §8(d) S1 names: 80 % inter blocks in inter
// frames, 40 % compound (average 50 / distance 20 / wedge 15 / difference-weighted 15), OBMC
// 10 %, local warp 5 %, uniform interpolation filters, motion vectors uniform within ±64 px
// at 1/8-pel (a target per coded vector: the difference to the predictor is what gets coded),
// loop-restoration unit types 50 / 50.
//
// Test and bench infrastructure: nothing in av1dec_amd/ links it.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "parser.h"

using namespace av1p;

extern "C" {
typedef struct av1bsw_params {
    int width, height;
    uint32_t seed;
    int sb128;             // 128x128 superblocks (else 64x64)
    int tile_cols_log2, tile_rows_log2;
    int base_q_idx;
    int key_interval;      // 0: key frame only at frame 0
    int lf_level[4], lf_sharpness;
    int lf_delta_update;   // write explicit loop-filter ref/mode delta updates
    int delta_q;           // 0 off, 1 delta_q_present, 2 + delta_lf_present, 3 + delta_lf_multi
    int gm;                // global motion: 0 identity, 1 translation, 2 rotzoom, 3 affine (+ rotzoom)
    int cdef;              // cdef_bits + 1 (0: CDEF strengths all zero)
    int lr;                // 0 none, 1 Wiener luma + self-guided chroma, 2 switchable on all planes
    int verify;            // re-parse every temporal unit and compare the batches
    int intra_only;        // every frame a key frame (intra)
    int hidden;            // hidden frames: every 4th unit after a key frame codes an ALTREF-style frame
                           // (show_frame = 0, two frames ahead, slot 7) before its shown frame, and
                           // two units later a show_existing_frame unit shows it
} av1bsw_params;
}

namespace {

// ---- od_ec range encoder (libaom od_ec_encode_q15 / od_ec_enc_done; the exact inverse of
// SymbolDecoder::read over CDFs in the inverted form) ----
struct RangeEncoder {
    std::vector<uint16_t> pre;  // output before carry propagation
    uint64_t low = 0;
    uint32_t rng = 0x8000;
    int cnt = -9;
    void reset()
    {
        pre.clear();
        low = 0;
        rng = 0x8000;
        cnt = -9;
    }
    static int ilog(uint32_t v)
    {
        int n = 0;
        while (v) n++, v >>= 1;
        return n;
    }
    void encode(const uint16_t* icdf, int s, int nsym)
    {
        const uint32_t fl = s > 0 ? icdf[s - 1] : 32768u, fh = icdf[s];
        const int N = nsym - 1;
        uint64_t l = low;
        uint32_t r = rng;
        if (fl < 32768u) {
            const uint32_t u = ((r >> 8) * (fl >> 6) >> 1) + 4u * (uint32_t)(N - (s - 1));
            const uint32_t v = ((r >> 8) * (fh >> 6) >> 1) + 4u * (uint32_t)(N - s);
            l += r - u;
            r = u - v;
        } else {
            r -= ((r >> 8) * (fh >> 6) >> 1) + 4u * (uint32_t)(N - s);
        }
        const int d = 16 - ilog(r);
        int c = cnt, sh = c + d;
        if (sh >= 0) {
            c += 16;
            uint64_t m = ((uint64_t)1 << c) - 1;
            if (sh >= 8) {
                pre.push_back((uint16_t)(l >> c));
                l &= m;
                c -= 8;
                m >>= 8;
            }
            pre.push_back((uint16_t)(l >> c));
            sh = c + d - 24;
            l &= m;
        }
        low = l << d;
        rng = r << d;
        cnt = sh;
    }
    std::vector<uint8_t> finish()
    {
        int c = cnt, s = c + 10;
        const uint64_t m = 0x3FFF;
        uint64_t e = ((low + m) & ~m) | (m + 1);
        if (s > 0) {
            uint64_t n = ((uint64_t)1 << (c + 16)) - 1;
            do {
                pre.push_back((uint16_t)(e >> (c + 16)));
                e &= n;
                s -= 8;
                c -= 8;
                n >>= 8;
            } while (s > 0);
        }
        std::vector<uint8_t> out(pre.size());
        uint32_t carry = 0;
        for (size_t i = pre.size(); i-- > 0;) {
            carry += pre[i];
            out[i] = (uint8_t)carry;
            carry >>= 8;
        }
        return out;
    }
};

// ---- MSB-first bit writer (the inverse of BitReader) ----
struct BitWriter {
    std::vector<uint8_t> b;
    size_t pos = 0;
    void put(int bit)
    {
        if (!(pos & 7)) b.push_back(0);
        if (bit) b.back() |= (uint8_t)(0x80 >> (pos & 7));
        pos++;
    }
    void f(int n, uint32_t v)
    {
        for (int i = n - 1; i >= 0; i--) put((v >> i) & 1);
    }
    void flag(bool v) { put(v); }
    void su(int n, int v) { f(n, (uint32_t)v & ((1u << n) - 1)); }
    void ns(uint32_t n, uint32_t v)  // ns(n) of spec 4.10.7
    {
        int w = 0;
        for (uint32_t x = n; x; x >>= 1) w++;
        const uint32_t m = (1u << w) - n;
        if (v < m) {
            f(w - 1, v);
        } else {
            f(w - 1, m + ((v - m) >> 1));
            f(1, (v - m) & 1);
        }
    }
    void align()
    {
        while (pos & 7) put(0);
    }
    void trailing()
    {
        put(1);
        align();
    }
};

// subexponential coding of the global motion parameters (inverse of obu.cpp decode_subexp /
// decode_signed_subexp_with_ref, spec 5.9.26-28)
static int recenter(int r, int v)
{
    if (v > 2 * r) return v;
    if (v >= r) return (v - r) << 1;
    return ((r - v) << 1) - 1;
}
static void encode_subexp(BitWriter& w, int numSyms, int v)
{
    int i = 0, mk = 0;
    const int k = 3;
    for (;;) {
        const int b2 = i ? k + i - 1 : k;
        const int a = 1 << b2;
        if (numSyms <= mk + 3 * a) {
            w.ns((uint32_t)(numSyms - mk), (uint32_t)(v - mk));
            return;
        }
        const bool more = v >= mk + a;
        w.flag(more);
        if (!more) {
            w.f(b2, (uint32_t)(v - mk));
            return;
        }
        i++;
        mk += a;
    }
}
static void encode_signed_subexp_with_ref(BitWriter& w, int low, int high, int r, int x)
{
    const int mx = high - low;
    r -= low;
    x -= low;
    const int v = (r << 1) <= mx ? recenter(r, x) : recenter(mx - 1 - r, mx - 1 - x);
    encode_subexp(w, mx, v);
}

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x2545F4914F6CDD1Dull) {}
    uint32_t next()
    {
        s ^= s >> 12;
        s ^= s << 25;
        s ^= s >> 27;
        return (uint32_t)((s * 0x2545F4914F6CDD1Dull) >> 32);
    }
    int uniform(int n) { return (int)(((uint64_t)next() * (uint32_t)n) >> 32); }
    int range(int lo, int hi) { return lo + uniform(hi - lo + 1); }
    bool bern(double p) { return next() < (uint32_t)(p * 4294967295.0); }
};

static void obu(std::vector<uint8_t>& out, int type, const std::vector<uint8_t>& payload)
{
    out.push_back((uint8_t)((type << 3) | 2));  // has_size_field
    uint64_t n = payload.size();
    do {
        uint8_t byte = n & 0x7f;
        n >>= 7;
        if (n) byte |= 0x80;
        out.push_back(byte);
    } while (n);
    out.insert(out.end(), payload.begin(), payload.end());
}

static bool same_frame(const Frame& a, const Frame& b, std::string& why)
{
    auto cmp = [&](const void* x, const void* y, size_t n, size_t m, const char* what) {
        if (n != m || (n && memcmp(x, y, n))) {
            why = what;
            return false;
        }
        return true;
    };
    return cmp(&a.hdr, &b.hdr, sizeof(a.hdr), sizeof(b.hdr), "header") &&
           cmp(a.mi.data(), b.mi.data(), a.mi.size() * sizeof(av1r_mi), b.mi.size() * sizeof(av1r_mi), "mi") &&
           cmp(a.blocks.data(), b.blocks.data(), a.blocks.size() * sizeof(av1r_block), b.blocks.size() * sizeof(av1r_block),
               "blocks") &&
           cmp(a.tbs.data(), b.tbs.data(), a.tbs.size() * sizeof(av1r_tb), b.tbs.size() * sizeof(av1r_tb), "tbs") &&
           cmp(a.coefs.data(), b.coefs.data(), a.coefs.size() * 4, b.coefs.size() * 4, "coefs") &&
           cmp(a.palette.data(), b.palette.data(), a.palette.size(), b.palette.size(), "palette") &&
           cmp(a.cdef.data(), b.cdef.data(), a.cdef.size(), b.cdef.size(), "cdef") &&
           cmp(a.lr.data(), b.lr.data(), a.lr.size() * sizeof(av1r_lr_unit), b.lr.size() * sizeof(av1r_lr_unit), "lr");
}

class Writer : public WriterHook {
public:
    av1bsw_params prm;
    Parser P;       // the walk that writes
    Parser V;       // an independent parse of the output (verify)
    RangeEncoder enc;
    Rng rng;
    Cdfs defaults;  // the distributions the chooser samples from
    int t = 0, since_key = 0;
    int coded_since_key = 0;  // coded shown frames since the key frame (the slot cycle)
    bool hidden_pending = false;  // slot 7 holds a hidden frame not yet shown
    int slot_of_age[8] = {};  // slot holding the frame `age` frames back (age 1..7)
    std::vector<uint8_t> tu;
    std::string err;
    int64_t symbols = 0;
    // motion vector plan: the difference the next read_mv codes
    int mv_diff[2] = {0, 0};

    explicit Writer(const av1bsw_params& p) : prm(p), rng(p.seed) {}

    int fail(const char* fmt, ...)
    {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        err = buf;
        return -1;
    }

    // ---- WriterHook ----
    void mv_pred(const Mv& pred, int /*ctx*/) override
    {
        const int R = 64 * 8;  // ±64 px in 1/8 pel
        const int tr = rng.range(-R, R), tc = rng.range(-R, R);
        mv_diff[0] = tr - pred.r;
        mv_diff[1] = tc - pred.c;
    }
    // Golomb codes of coefficient levels: the prefix ends by its 4th bit (levels below 30 above
    // the base range), as coded levels stay in real streams -- random prefixes reach lengths
    // that overflow the reference's int16 levels (TransformBlock.cpp:1620-1635)
    int force_bit = -1;
    void golomb_prefix(int length) override { force_bit = length >= 4 ? 1 : -1; }
    int symbol(uint16_t* cdf, int nsym) override
    {
        const int s = choose(cdf, nsym);
        if (s < 0 || s >= nsym) {
            if (err.empty()) fail("chooser produced symbol %d of %d", s, nsym);
            enc.encode(cdf, 0, nsym);
            return 0;
        }
        enc.encode(cdf, s, nsym);
        symbols++;
        return s;
    }

    int sample(const uint16_t* icdf, int nsym)
    {
        const uint32_t u = rng.next() & 32767;
        for (int s = 0; s < nsym - 1; s++)
            if (u < 32768u - icdf[s]) return s;
        return nsym - 1;
    }
    template <class T>
    bool in(const uint16_t* p, const T& field) const
    {
        return (const uint8_t*)p >= (const uint8_t*)&field && (const uint8_t*)p < (const uint8_t*)&field + sizeof(field);
    }
    int mv_symbol(const uint16_t* p, int nsym)
    {
        const MvCdfs& m = P.tile.tcdf.mv[0];
        if (p == m.joints) return (mv_diff[0] != 0) * 2 + (mv_diff[1] != 0);
        for (int k = 0; k < 2; k++) {
            const MvComp& c = m.comp[k];
            if (!in(p, c)) continue;
            const int d = mv_diff[k];
            const int mag = d < 0 ? -d : d;
            const int v = mag - 1;  // >= 0: a zero component is never read
            int cls = 0;
            if (v >= 16) {
                cls = 1;
                while (cls < 10 && v >= (16 << cls)) cls++;
            }
            const int rem = cls ? v - (8 << cls) : v;  // (d << 3) | (fr << 1) | hp
            if (p == c.sign) return d < 0;
            if (p == c.classes) return cls;
            if (p == c.class0) return rem >> 3;
            if (in(p, c.class0_fp) || p == c.fp) return (rem >> 1) & 3;
            if (p == c.class0_hp || p == c.hp) return rem & 1;
            for (int i = 0; i < 10; i++)
                if (p == c.bits[i]) return (rem >> (3 + i)) & 1;
        }
        (void)nsym;
        fail("unexpected motion vector CDF");
        return 0;
    }
    int choose(uint16_t* cdf, int nsym)
    {
        const uint8_t* base = (const uint8_t*)&P.tile.tcdf;
        const ptrdiff_t off = (const uint8_t*)cdf - base;
        if (off < 0 || off >= (ptrdiff_t)sizeof(Cdfs)) {  // literal bits, derived CDFs
            if (force_bit >= 0) {
                const int b = force_bit;
                force_bit = -1;
                return b;
            }
            return sample(cdf, nsym);
        }
        const ModeCdfs& M = P.tile.tcdf.mode;
        if (in(cdf, P.tile.tcdf.mv[0])) return mv_symbol(cdf, nsym);
        if (in(cdf, M.intra_inter)) return rng.bern(0.8);
        if (in(cdf, M.comp_inter)) return rng.bern(0.4);
        if (in(cdf, M.comp_group_idx)) return rng.bern(0.3);      // wedge + difference-weighted
        if (in(cdf, M.compound_index)) return rng.bern(5.0 / 7);  // 1: average, 0: distance
        if (in(cdf, M.compound_type)) return rng.bern(0.5);       // 0: wedge, 1: difference-weighted
        if (in(cdf, M.motion_mode)) {
            const uint32_t u = rng.next() % 100;
            return u < 85 ? 0 : u < 95 ? 1 : 2;  // simple / OBMC / local warp
        }
        if (in(cdf, M.obmc)) return rng.bern(0.1);
        if (in(cdf, M.switchable_interp)) return rng.uniform(3);
        if (in(cdf, M.wiener_restore) || in(cdf, M.sgrproj_restore)) return rng.bern(0.5);
        if (in(cdf, M.partition)) {
            // the synthetic batch generator's block-size mix (tools/synth/synth.cpp partition()):
            // split 85 % above 32x32, 55 % at 32x32, 35 % at 16x16, 25 % at 8x8; otherwise
            // NONE 60 %, HORZ / VERT 20 %, HORZ_4 / VERT_4 20 % where they exist
            const int bsl = (int)((off - ((const uint8_t*)M.partition - base)) / sizeof(M.partition[0])) / 4;  // 8x8 .. 128x128
            const int pSplit = bsl >= 3 ? 85 : bsl == 2 ? 55 : bsl == 1 ? 35 : 25;
            if ((int)(rng.next() % 100) < pSplit) return PARTITION_SPLIT;
            const int u = (int)(rng.next() % 100);
            if (u < 60) return PARTITION_NONE;
            if (u < 80 || nsym < 10) return rng.bern(0.5) ? PARTITION_HORZ : PARTITION_VERT;
            return rng.bern(0.5) ? PARTITION_HORZ_4 : PARTITION_VERT_4;
        }
        return sample((const uint16_t*)((const uint8_t*)&defaults + off), nsym);
    }

    // ---- headers ----
    std::vector<uint8_t> sequence_header()
    {
        BitWriter w;
        w.f(3, 0);   // seq_profile (8-bit 4:2:0)
        w.f(1, 0);   // still_picture
        w.f(1, 0);   // reduced_still_picture_header
        w.f(1, 0);   // timing_info_present_flag
        w.f(1, 0);   // initial_display_delay_present_flag
        w.f(5, 0);   // operating_points_cnt_minus_1
        w.f(12, 0);  // operating_point_idc[0]
        const int level = prm.width * prm.height > 2048 * 1152 ? 12 : 8;  // 5.0 / 4.0
        w.f(5, (uint32_t)level);
        if (level > 7) w.f(1, 0);  // seq_tier
        auto bits = [](int v) {
            int n = 1;
            while ((1 << n) < v) n++;
            return n;
        };
        const int wb = bits(prm.width), hb = bits(prm.height);
        w.f(4, (uint32_t)(wb - 1));
        w.f(4, (uint32_t)(hb - 1));
        w.f(wb, (uint32_t)(prm.width - 1));
        w.f(hb, (uint32_t)(prm.height - 1));
        w.f(1, 0);  // frame_id_numbers_present_flag
        w.f(1, (uint32_t)!!prm.sb128);
        w.f(1, 1);  // enable_filter_intra
        w.f(1, 1);  // enable_intra_edge_filter
        w.f(1, 1);  // enable_interintra_compound
        w.f(1, 1);  // enable_masked_compound
        w.f(1, 1);  // enable_warped_motion
        w.f(1, 1);  // enable_dual_filter
        w.f(1, 1);  // enable_order_hint
        w.f(1, 1);  // enable_jnt_comp
        w.f(1, 1);  // enable_ref_frame_mvs
        w.f(1, 0);  // seq_choose_screen_content_tools
        w.f(1, 0);  // seq_force_screen_content_tools
        w.f(3, 6);  // order_hint_bits_minus_1
        w.f(1, 0);  // enable_superres
        w.f(1, 1);  // enable_cdef
        w.f(1, 1);  // enable_restoration
        w.f(1, 0);  // high_bitdepth
        w.f(1, 0);  // mono_chrome
        w.f(1, 0);  // color_description_present_flag
        w.f(1, 0);  // color_range
        w.f(2, 0);  // chroma_sample_position
        w.f(1, 0);  // separate_uv_delta_q
        w.f(1, 0);  // film_grain_params_present
        w.trailing();
        return w.b;
    }

    // the frame header; `key` frames refresh every slot, inter frames one slot, referencing
    // the seven most recent frames (the key frame in slot 0 as GOLDEN)
    // (show = false: a hidden, showable frame whose order hint is `hint_ahead` units ahead)
    void frame_header(BitWriter& w, bool key, int refresh, const int* ref_idx, bool show = true, int hint_ahead = 0)
    {
        const SeqHdr& seq = P.seq;
        w.f(1, 0);  // show_existing_frame
        w.f(2, key ? KEY_FRAME : INTER_FRAME);
        w.f(1, show);  // show_frame
        if (!show) w.f(1, 1);  // showable_frame
        if (!key) w.f(1, 0);  // error_resilient_mode
        w.f(1, 0);  // disable_cdf_update
        w.f(1, 0);  // frame_size_override_flag
        const int hint = (t + hint_ahead) & ((1 << seq.order_hint_bits) - 1);
        w.f(seq.order_hint_bits, (uint32_t)hint);
        if (!key) w.f(3, 0);  // primary_ref_frame = LAST
        if (!key) w.f(8, (uint32_t)refresh);
        if (key) {
            w.f(1, 0);  // render_and_frame_size_different
        } else {
            w.f(1, 0);  // frame_refs_short_signaling
            for (int i = 0; i < kRefsPerFrame; i++) w.f(3, (uint32_t)ref_idx[i]);
            w.f(1, 0);  // render_and_frame_size_different
            w.f(1, 1);  // allow_high_precision_mv
            w.f(1, 1);  // is_filter_switchable
            w.f(1, 1);  // is_motion_mode_switchable
            w.f(1, 1);  // use_ref_frame_mvs
        }
        w.f(1, 0);  // disable_frame_end_update_cdf
        // tile_info: uniform spacing
        {
            auto tile_log2 = [](int blk, int target) {
                int k = 0;
                while ((blk << k) < target) k++;
                return k;
            };
            const int miCols = 2 * ((prm.width + 7) >> 3), miRows = 2 * ((prm.height + 7) >> 3);
            const int sbCols = prm.sb128 ? (miCols + 31) >> 5 : (miCols + 15) >> 4;
            const int sbRows = prm.sb128 ? (miRows + 31) >> 5 : (miRows + 15) >> 4;
            const int sbSize = prm.sb128 ? 7 : 6;
            const int minLog2TileCols = tile_log2(4096 >> sbSize, sbCols);
            const int maxLog2TileCols = tile_log2(1, std::min(sbCols, 64));
            const int maxLog2TileRows = tile_log2(1, std::min(sbRows, 64));
            const int minLog2Tiles = std::max(minLog2TileCols, tile_log2((4096 * 2304) >> (2 * sbSize), sbRows * sbCols));
            const int cols = std::min(std::max(prm.tile_cols_log2, minLog2TileCols), maxLog2TileCols);
            w.f(1, 1);
            for (int i = minLog2TileCols; i < cols; i++) w.f(1, 1);
            if (cols < maxLog2TileCols) w.f(1, 0);
            const int minLog2TileRows = std::max(minLog2Tiles - cols, 0);
            const int rows = std::min(std::max(prm.tile_rows_log2, minLog2TileRows), maxLog2TileRows);
            for (int i = minLog2TileRows; i < rows; i++) w.f(1, 1);
            if (rows < maxLog2TileRows) w.f(1, 0);
            if (cols + rows > 0) {
                w.f(cols + rows, (uint32_t)((cols + rows) ? rng.uniform(1 << (cols + rows)) : 0));  // context_update_tile_id
                w.f(2, 3);  // tile_size_bytes_minus_1
            }
        }
        // quantization_params
        w.f(8, (uint32_t)prm.base_q_idx);
        w.f(1, 0);  // delta_coded (DeltaQYDc)
        w.f(1, 0);  // DeltaQUDc
        w.f(1, 0);  // DeltaQUAc
        w.f(1, 0);  // using_qmatrix
        w.f(1, 0);  // segmentation_enabled
        if (prm.base_q_idx > 0) {
            w.f(1, prm.delta_q > 0);
            if (prm.delta_q > 0) {
                w.f(2, 1);  // delta_q_res (log2)
                w.f(1, prm.delta_q > 1);
                if (prm.delta_q > 1) {
                    w.f(2, 0);  // delta_lf_res
                    w.f(1, prm.delta_q > 2);
                }
            }
        }
        // loop_filter_params
        w.f(6, (uint32_t)prm.lf_level[0]);
        w.f(6, (uint32_t)prm.lf_level[1]);
        if (prm.lf_level[0] || prm.lf_level[1]) {
            w.f(6, (uint32_t)prm.lf_level[2]);
            w.f(6, (uint32_t)prm.lf_level[3]);
        }
        w.f(3, (uint32_t)prm.lf_sharpness);
        w.f(1, 1);  // loop_filter_delta_enabled
        w.f(1, (uint32_t)!!prm.lf_delta_update);
        if (prm.lf_delta_update) {
            for (int i = 0; i < 8; i++) {
                const bool upd = rng.bern(0.5);
                w.f(1, upd);
                if (upd) w.su(7, rng.range(-20, 20));
            }
            for (int i = 0; i < 2; i++) {
                const bool upd = rng.bern(0.5);
                w.f(1, upd);
                if (upd) w.su(7, rng.range(-20, 20));
            }
        }
        // cdef_params
        w.f(2, (uint32_t)rng.uniform(4));  // cdef_damping_minus_3
        const int cdefBits = prm.cdef > 0 ? prm.cdef - 1 : 0;
        w.f(2, (uint32_t)cdefBits);
        for (int i = 0; i < (1 << cdefBits); i++) {
            const bool on = prm.cdef > 0;
            w.f(4, on ? (uint32_t)rng.uniform(16) : 0);
            w.f(2, on ? (uint32_t)rng.uniform(4) : 0);
            w.f(4, on ? (uint32_t)rng.uniform(16) : 0);
            w.f(2, on ? (uint32_t)rng.uniform(4) : 0);
        }
        // lr_params: 0 NONE, 1 SWITCHABLE, 2 WIENER, 3 SGRPROJ (coded values)
        {
            const int types[3] = {prm.lr == 1 ? 2 : prm.lr == 2 ? 1 : 0, prm.lr == 1 ? 3 : prm.lr == 2 ? 1 : 0,
                                  prm.lr == 1 ? 3 : prm.lr == 2 ? 1 : 0};
            for (int i = 0; i < 3; i++) w.f(2, (uint32_t)types[i]);
            if (prm.lr) {
                int s;  // luma unit 64 << s
                if (prm.sb128) {
                    s = 1 + rng.uniform(2);  // 128 or 256
                    w.f(1, (uint32_t)(s - 1));
                } else {
                    s = rng.uniform(3);  // 64, 128 or 256
                    w.f(1, s > 0);
                    if (s > 0) w.f(1, s > 1);
                }
                // lr_uv_shift; never 32-px chroma units: the reference corrupts memory on
                // them (SIGFPE / SIGSEGV at -O1)
                w.f(1, s > 0 ? (uint32_t)rng.uniform(2) : 0);
            }
        }
        w.f(1, 1);  // tx_mode_select
        if (!key) {
            w.f(1, 1);  // reference_select
            // skip_mode_present when skipModeAllowed (spec 5.9.22): a forward reference and a
            // backward one, or two forward references with different hints
            const int bits = seq.order_hint_bits, cur = hint;
            auto dist = [&](int a, int b) {
                const int m = 1 << (bits - 1);
                int d = a - b;
                return (d & (m - 1)) - (d & m);
            };
            int fwd = -1, bwd = -1, fwdHint = 0, bwdHint = 0;
            for (int i = 0; i < kRefsPerFrame; i++) {
                const int h = P.slots[ref_idx[i]].order_hint;
                if (dist(h, cur) < 0) {
                    if (fwd < 0 || dist(h, fwdHint) > 0) fwd = i, fwdHint = h;
                } else if (dist(h, cur) > 0) {
                    if (bwd < 0 || dist(h, bwdHint) < 0) bwd = i, bwdHint = h;
                }
            }
            bool allowed = fwd >= 0 && bwd >= 0;
            if (fwd >= 0 && bwd < 0)
                for (int i = 0; i < kRefsPerFrame && !allowed; i++) {
                    const int h = P.slots[ref_idx[i]].order_hint;
                    if (dist(h, fwdHint) < 0) allowed = true;
                }
            if (allowed) w.f(1, rng.bern(0.5));
            w.f(1, 1);  // allow_warped_motion
        }
        w.f(1, 0);  // reduced_tx_set
        if (!key) {
            // global_motion_params against the primary reference frame's parameters
            const RefSlot& pr = P.slots[ref_idx[0]];
            for (int ref = LAST_FRAME; ref <= ALTREF_FRAME; ref++) {
                int type = AV1R_GM_IDENTITY;
                if (prm.gm == 1 && ref == LAST_FRAME) type = AV1R_GM_TRANSLATION;
                if (prm.gm >= 2 && (ref == LAST_FRAME || ref == GOLDEN_FRAME)) type = AV1R_GM_ROTZOOM;
                if (prm.gm == 3 && ref == LAST_FRAME) type = AV1R_GM_AFFINE;
                w.f(1, type != AV1R_GM_IDENTITY);
                if (type != AV1R_GM_IDENTITY) {
                    w.f(1, type == AV1R_GM_ROTZOOM);
                    if (type != AV1R_GM_ROTZOOM) w.f(1, type == AV1R_GM_TRANSLATION);
                }
                auto param = [&](int idx) {
                    int absBits = 12, precBits = 15;
                    if (idx < 2) {
                        absBits = type == AV1R_GM_TRANSLATION ? 9 : 12;  // allow_high_precision_mv = 1
                        precBits = type == AV1R_GM_TRANSLATION ? 3 : 6;
                    }
                    const int precDiff = kWarpPrecBits - precBits;
                    const int sub = (idx % 3) == 2 ? (1 << precBits) : 0;
                    const int mx = 1 << absBits;
                    const int r = (pr.saved_gm[ref][idx] >> precDiff) - sub;
                    // small motions: +-8 px translation, +-1 % zoom / rotation terms
                    const int lim = idx < 2 ? (type == AV1R_GM_TRANSLATION ? 64 : 512) : 300;
                    const int x = rng.range(-lim, lim);
                    encode_signed_subexp_with_ref(w, -mx, mx + 1, r, x);
                };
                if (type >= AV1R_GM_ROTZOOM) {
                    param(2);
                    param(3);
                    if (type == AV1R_GM_AFFINE) {
                        param(4);
                        param(5);
                    }
                }
                if (type >= AV1R_GM_TRANSLATION) {
                    param(0);
                    param(1);
                }
            }
        }
    }

    void set_defaults()
    {
        const int q = prm.base_q_idx;
        defaults.coef = kDefaultCoefCdfs[q <= 20 ? 0 : q <= 60 ? 1 : q <= 120 ? 2 : 3];
        defaults.mode = kDefaultModeCdfs;
        defaults.mv[0] = kDefaultMvCdfs[0];
        defaults.mv[1] = kDefaultMvCdfs[1];
    }

    // one temporal unit: temporal delimiter, (sequence header,) one shown frame
    int next()
    {
        tu.clear();
        err.clear();
        const bool key = prm.intra_only || t == 0 || (prm.key_interval > 0 && t % prm.key_interval == 0);
        std::vector<uint8_t> seqObu;
        tu.push_back((uint8_t)(OBU_TEMPORAL_DELIMITER << 3 | 2));
        tu.push_back(0);
        if (t == 0) {
            set_defaults();
            const std::vector<uint8_t> sh = sequence_header();
            obu(tu, OBU_SEQUENCE_HEADER, sh);
            BitReader br(sh.data(), sh.size());
            if (P.parse_sequence_header(br)) return fail("sequence header: %s", P.err.c_str());
        }
        int refIdx[7] = {}, refresh = 0xff;
        const bool hid = prm.hidden && !key;
        if (key) {
            since_key = 0;
            coded_since_key = 0;
            hidden_pending = false;
            for (int a = 0; a < 8; a++) slot_of_age[a] = 0;
        } else {
            since_key++;
            if (hid && since_key % 4 == 3 && hidden_pending) {
                // a show_existing_frame unit: the hidden frame of two units back (its order hint
                // is this unit's), spec 5.9.2 / 7.21 (Av1Decoder.cpp:158-169)
                BitWriter sw;
                sw.f(1, 1);  // show_existing_frame
                sw.f(3, 7);  // frame_to_show_map_idx
                sw.trailing();
                BitReader br(sw.b.data(), sw.b.size());
                P.seen_frame_header = false;
                if (P.parse_frame_header(br)) return fail("unit %d: show_existing header: %s", t, P.err.c_str());
                obu(tu, OBU_FRAME_HEADER, sw.b);
                hidden_pending = false;
                return end_unit();
            }
            coded_since_key++;
            // this frame's slot: cycle 1..7 (slot 0 keeps the key frame as GOLDEN); with hidden
            // frames 1..6, and ALTREF is slot 7 (the latest hidden frame, or the key frame)
            const int nslots = hid ? 6 : 7;
            const int slot = 1 + (coded_since_key - 1) % nslots;
            refresh = 1 << slot;
            const int ages[7] = {1, 2, 3, 0, 4, 5, 6};  // LAST, LAST2, LAST3, GOLDEN(key), BWDREF, ALTREF2, ALTREF
            for (int i = 0; i < 7; i++) refIdx[i] = ages[i] == 0 ? 0 : slot_of_age[ages[i]];
            if (hid) refIdx[6] = 7;
            for (int a = 7; a > 1; a--) slot_of_age[a] = slot_of_age[a - 1];
            slot_of_age[1] = slot;
            if (hid && since_key % 4 == 1) {
                // a hidden frame first (two units ahead, into slot 7), shown two units later
                BitWriter hh;
                frame_header(hh, false, 1 << 7, refIdx, false, 2);
                if (int rc = code_frame(hh)) return rc;
                hidden_pending = true;
            }
        }
        if (key) slot_of_age[1] = 0;
        BitWriter hw;
        frame_header(hw, key, refresh, refIdx);
        if (int rc = code_frame(hw)) return rc;
        return end_unit();
    }

    // the frame whose uncompressed header is in hw: header check, tiles, one OBU_FRAME
    int code_frame(BitWriter& hw)
    {
        const size_t hdrBits = hw.pos;
        {
            std::vector<uint8_t> hb = hw.b;
            hb.resize(hb.size() + 8, 0);  // the parser may look ahead; the bit count is checked
            BitReader br(hb.data(), hb.size());
            if (P.parse_frame_header(br)) return fail("frame %d header: %s", t, P.err.c_str());
            if (br.pos != hdrBits) return fail("frame %d header: parsed %zu bits of %zu written", t, br.pos, hdrBits);
        }
        hw.align();
        const int numTiles = P.fh.tile_cols * P.fh.tile_rows;
        if (numTiles > 1) {
            hw.f(1, 0);  // tile_start_and_end_present_flag
            hw.align();
        }
        std::vector<uint8_t> payload = hw.b;
        for (int tn = 0; tn < numTiles; tn++) {
            static const uint8_t none = 0;
            P.begin_tile(P.tile, tn, &none, 0);
            P.tile.sd.hook = this;
            enc.reset();
            const int rc = P.decode_tile(P.tile);
            P.tile.sd.hook = nullptr;
            P.merge_tile(P.tile, tn);
            if (rc || !err.empty()) return fail("frame %d tile %d: %s", t, tn, err.empty() ? P.err.c_str() : err.c_str());
            std::vector<uint8_t> data = enc.finish();
            if (data.empty()) data.push_back(0);
            if (tn + 1 < numTiles) {
                const uint32_t sz = (uint32_t)data.size() - 1;
                for (int i = 0; i < 4; i++) payload.push_back((uint8_t)(sz >> (8 * i)));
            }
            payload.insert(payload.end(), data.begin(), data.end());
            P.tile_num = tn + 1;
        }
        if (P.finish_frame()) return fail("frame %d: %s", t, P.err.c_str());
        P.seen_frame_header = false;
        obu(tu, OBU_FRAME, payload);
        return 0;
    }

    // verify the unit (every frame it carries re-parsed and compared) and advance
    int end_unit()
    {
        int rc = 0;
        if (prm.verify) {
            if (V.decode_tu(tu.data(), tu.size())) {
                rc = fail("frame %d: the written unit does not parse: %s", t, V.err.c_str());
            } else if (V.done.size() != P.done.size()) {
                rc = fail("frame %d: parsed %zu frames, wrote %zu", t, V.done.size(), P.done.size());
            } else {
                for (size_t i = 0; i < V.done.size() && !rc; i++) {
                    std::string why;
                    if (!same_frame(*V.done[i], *P.done[i], why)) rc = fail("frame %d: parsed batch differs (%s)", t, why.c_str());
                }
            }
            for (auto* f : V.done) delete f;
            V.done.clear();
        }
        for (auto* f : P.done) delete f;
        P.done.clear();
        t++;
        return rc;
    }
};

}  // namespace

extern "C" {

void* av1bsw_open(const av1bsw_params* p)
{
    if (!p || p->width < 16 || p->height < 16 || (p->width & 1) || (p->height & 1) || p->base_q_idx < 1 ||
        p->base_q_idx > 255)
        return nullptr;
    return new Writer(*p);
}

// the next temporal unit (valid until the next call); 0 or -1 (av1bsw_error says why)
int av1bsw_next(void* h, const uint8_t** data, size_t* size)
{
    Writer* w = (Writer*)h;
    const int rc = w->next();
    *data = w->tu.data();
    *size = w->tu.size();
    return rc;
}

const char* av1bsw_error(void* h) { return ((Writer*)h)->err.c_str(); }
int64_t av1bsw_symbols(void* h) { return ((Writer*)h)->symbols; }
void av1bsw_close(void* h) { delete (Writer*)h; }

}  // extern "C"

#ifdef AV1BSW_MAIN
// av1bsw -o out.ivf [-w 1920] [-h 1080] [-n 60] [-s seed] [--tiles C R] [--sb64] [-q 96]
//        [--sharp N] [--lf-deltas] [--delta-q N] [--gm N] [--cdef N] [--lr N] [--key N] [--hidden] [--verify]
int main(int argc, char** argv)
{
    av1bsw_params p = {};
    p.width = 1920;
    p.height = 1080;
    p.seed = 0x5EED0001;
    p.sb128 = 1;
    p.base_q_idx = 96;
    p.lf_level[0] = 32, p.lf_level[1] = 32, p.lf_level[2] = 16, p.lf_level[3] = 16;
    p.cdef = 4;
    p.lr = 1;
    int n = 60;
    const char* out = nullptr;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto arg = [&]() { return i + 1 < argc ? argv[++i] : (fprintf(stderr, "%s needs a value\n", a.c_str()), exit(2), ""); };
        if (a == "-o") out = arg();
        else if (a == "-w") p.width = atoi(arg());
        else if (a == "-h") p.height = atoi(arg());
        else if (a == "-n") n = atoi(arg());
        else if (a == "-s") p.seed = (uint32_t)strtoul(arg(), nullptr, 0);
        else if (a == "-q") p.base_q_idx = atoi(arg());
        else if (a == "--tiles") { p.tile_cols_log2 = atoi(arg()); p.tile_rows_log2 = atoi(arg()); }
        else if (a == "--sb64") p.sb128 = 0;
        else if (a == "--sharp") p.lf_sharpness = atoi(arg());
        else if (a == "--lf-deltas") p.lf_delta_update = 1;
        else if (a == "--delta-q") p.delta_q = atoi(arg());
        else if (a == "--gm") p.gm = atoi(arg());
        else if (a == "--cdef") p.cdef = atoi(arg());
        else if (a == "--lr") p.lr = atoi(arg());
        else if (a == "--key") p.key_interval = atoi(arg());
        else if (a == "--intra") p.intra_only = 1;
        else if (a == "--hidden") p.hidden = 1;
        else if (a == "--verify") p.verify = 1;
        else { fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
    }
    if (!out) { fprintf(stderr, "usage: av1bsw -o out.ivf [options]\n"); return 2; }
    void* h = av1bsw_open(&p);
    if (!h) { fprintf(stderr, "bad parameters\n"); return 2; }
    FILE* f = fopen(out, "wb");
    if (!f) { perror(out); return 1; }
    // IVF file header (tests/DecodeInput.cpp:187-254 reads it)
    uint8_t hdr[32] = {'D', 'K', 'I', 'F', 0, 0, 32, 0, 'A', 'V', '0', '1'};
    auto le16 = [](uint8_t* d, int v) { d[0] = (uint8_t)v; d[1] = (uint8_t)(v >> 8); };
    auto le32 = [](uint8_t* d, uint32_t v) { for (int i = 0; i < 4; i++) d[i] = (uint8_t)(v >> (8 * i)); };
    le16(hdr + 12, p.width);
    le16(hdr + 14, p.height);
    le32(hdr + 16, 30);
    le32(hdr + 20, 1);
    le32(hdr + 24, (uint32_t)n);
    fwrite(hdr, 1, 32, f);
    for (int i = 0; i < n; i++) {
        const uint8_t* d;
        size_t sz;
        if (av1bsw_next(h, &d, &sz)) { fprintf(stderr, "av1bsw: %s\n", av1bsw_error(h)); return 1; }
        uint8_t fh[12] = {};
        le32(fh, (uint32_t)sz);
        le32(fh + 4, (uint32_t)i);
        fwrite(fh, 1, 12, f);
        fwrite(d, 1, sz, f);
    }
    fclose(f);
    av1bsw_close(h);
    return 0;
}
#endif
