// refdump -- oracle harness (test infrastructure, this container only).
//
// Drives the REFERENCE decoder (oddstone/av1dec, built from its own sources into
// oracle/_ref/libref.a) over an IVF stream and, for every decoded frame, serialises
//   * the av1r frame batch (include/av1r.h) read out of the reference's parsed
//     SuperBlock -> Partition -> Block -> TransformBlock trees, exactly as the
//     reference's Decoder::decodeFrame (decoder/Av1Decoder.cpp:128-156) walks them, and
//   * the MD5 of the visible I420 planes after each reference stage: reconstruction
//     (Tile::decode), LoopFilter::filter, Cdef::filter, LoopRestoration::filter
//     (decode_frame_wrapup, Av1Decoder.cpp:171-192), and of the shown output.
// The decode loop mirrors Decoder::decode (Av1Decoder.cpp:49-109) so that the harness can
// observe the trees between parse and reconstruction.  Private members are reached with
// g++ -fno-access-control; nothing here changes what the reference computes.
//
// usage: refdump in.ivf out.av1b out.hashes
#include "Av1Decoder.h"
#include "BitReader.h"
#include "Block.h"
#include "Cdef.h"
#include "IntraPredict.h"
#include "LoopFilter.h"
#include "LoopRestoration.h"
#include "Parser.h"
#include "Partition.h"
#include "SuperBlock.h"
#include "Tile.h"
#include "TransformBlock.h"
#include "VideoFrame.h"
extern "C" {
#include "md5.h"
}
#include "av1r.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace YamiAv1;
using Yami::YuvFrame;

namespace {

std::string md5_planes(const YuvFrame& f)
{
    MD5_CTX ctx;
    MD5_Init(&ctx);
    for (int p = 0; p < 3; p++) {
        int w = p ? f.width >> 1 : f.width;
        int h = p ? f.height >> 1 : f.height;
        for (int y = 0; y < h; y++)
            MD5_Update(&ctx, f.data[p] + y * f.strides[p], w);
    }
    unsigned char d[16];
    MD5_Final(d, &ctx);
    static const char hex[] = "0123456789abcdef";
    std::string s;
    for (int i = 0; i < 16; i++) {
        s.push_back(hex[d[i] >> 4]);
        s.push_back(hex[d[i] & 15]);
    }
    return s;
}

struct Batch {
    av1r_frame_hdr hdr;
    std::vector<av1r_mi> mi;
    std::vector<av1r_block> blocks;
    std::vector<av1r_tb> tbs;
    std::vector<uint32_t> coefs;
    std::vector<uint8_t> palette;
    std::vector<int8_t> cdef;
    std::vector<av1r_lr_unit> lr;
};

template <class T>
void put_section(std::vector<uint8_t>& out, const T* data, size_t count)
{
    uint32_t n = (uint32_t)(count * sizeof(T));
    const uint8_t* b = (const uint8_t*)&n;
    out.insert(out.end(), b, b + 4);
    const uint8_t* d = (const uint8_t*)data;
    out.insert(out.end(), d, d + n);
    while (out.size() & 3)
        out.push_back(0);
}

void write_batch(FILE* fp, const Batch& b)
{
    std::vector<uint8_t> rec;
    put_section(rec, &b.hdr, 1);
    put_section(rec, b.mi.data(), b.mi.size());
    put_section(rec, b.blocks.data(), b.blocks.size());
    put_section(rec, b.tbs.data(), b.tbs.size());
    put_section(rec, b.coefs.data(), b.coefs.size());
    put_section(rec, b.palette.data(), b.palette.size());
    put_section(rec, b.cdef.data(), b.cdef.size());
    put_section(rec, b.lr.data(), b.lr.size());
    uint32_t magic = 0x454d5246; // "FRME"
    uint32_t len = (uint32_t)rec.size();
    fwrite(&magic, 4, 1, fp);
    fwrite(&len, 4, 1, fp);
    fwrite(rec.data(), 1, rec.size(), fp);
}

struct Dumper {
    Decoder dec;
    FILE* out = nullptr;
    FILE* hashes = nullptr;
    int frameNo = 0;
    Batch cur;
    MD5_CTX outCtx;

    // ---- per block (Block::decode, Block.cpp:1600-1608) ----
    void dumpBlock(Block& b, std::shared_ptr<YuvFrame>& frame)
    {
        const SequenceHeader& s = b.m_sequence;
        av1r_block r;
        memset(&r, 0, sizeof(r));
        r.mi_row = b.MiRow;
        r.mi_col = b.MiCol;
        r.mi_size = b.MiSize;
        r.qindex = (uint8_t)b.m_frame.get_qindex(b.CurrentQIndex, b.segment_id);
        r.y_mode = b.YMode;
        // only the fields the reference reads for this kind of block: UVMode, use_filter_intra
        // and CflAlpha* are uninitialised members of Block otherwise
        r.uv_mode = (b.HasChroma && !b.is_inter) ? b.UVMode : 0;
        r.angle_delta_y = b.AngleDeltaY;
        r.angle_delta_uv = b.AngleDeltaUV;
        r.filter_intra_mode = (!b.is_inter && b.use_filter_intra) ? b.filter_intra_mode : 0;
        if (!b.is_inter && b.HasChroma && b.UVMode == UV_CFL_PRED) {
            r.cfl_alpha_u = b.CflAlphaU;
            r.cfl_alpha_v = b.CflAlphaV;
        }
        r.palette_size_y = b.PaletteSizeY;
        r.palette_size_uv = b.PaletteSizeUV;
        uint32_t f = 0;
        if (b.is_inter) {
            f |= AV1R_BLK_INTER;
            r.motion_mode = b.motion_mode;
            r.compound_type = b.compound_type;
            r.interintra_mode = (b.interintra && !b.use_intrabc) ? b.interintra_mode : 0;
            // only the fields the reference reads for this compound type (others may be
            // uninitialised members of Block)
            if (b.compound_type == COMPOUND_WEDGE) {
                r.wedge_index = b.wedge_index;
                r.wedge_sign = b.wedge_sign;
            }
            if (b.compound_type == COMPOUND_DIFFWTD)
                r.mask_type = b.mask_type;
            if (b.interintra && !b.use_intrabc)
                f |= AV1R_BLK_INTERINTRA;
            if (b.interintra && !b.use_intrabc && b.wedge_interintra)
                f |= AV1R_BLK_WEDGE_II;
        }
        if (b.use_intrabc)
            f |= AV1R_BLK_INTRABC;
        if (b.Lossless)
            f |= AV1R_BLK_LOSSLESS;
        if (b.HasChroma)
            f |= AV1R_BLK_HAS_CHROMA;
        if (!b.is_inter && b.use_filter_intra)
            f |= AV1R_BLK_FILTER_INTRA;
        if (b.AvailL)
            f |= AV1R_BLK_AVAIL_L;
        if (b.AvailU)
            f |= AV1R_BLK_AVAIL_U;
        if (b.AvailLChroma)
            f |= AV1R_BLK_AVAIL_L_UV;
        if (b.AvailUChroma)
            f |= AV1R_BLK_AVAIL_U_UV;
        if (b.skip)
            f |= AV1R_BLK_SKIP;
        if (!b.is_inter) {
            std::vector<std::vector<uint8_t>> dummy;
            for (int plane = 0; plane < 2; plane++) {
                Block::IntraPredict ip(b, frame, plane, 0, 0, 2, 2, dummy);
                if (ip.getAboveSmooth())
                    f |= plane ? AV1R_BLK_SMOOTH_A_UV : AV1R_BLK_SMOOTH_A_Y;
                if (ip.getLeftSmooth())
                    f |= plane ? AV1R_BLK_SMOOTH_L_UV : AV1R_BLK_SMOOTH_L_Y;
            }
        }
        // block-level interintra edge flags (Block.cpp:128-133), read before prediction.
        bool isII = b.is_inter && b.RefFrame[1] == INTRA_FRAME;
        if (isII) {
            int sbRow = b.MiRow & b.sbMask, sbCol = b.MiCol & b.sbMask;
            for (int plane = 0; plane < 1 + b.HasChroma * 2; plane++) {
                int planeSz = b.get_plane_residual_size(b.MiSize, plane);
                int n4w = Num_4x4_Blocks_Wide[planeSz], n4h = Num_4x4_Blocks_High[planeSz];
                int subX = plane ? s.subsampling_x : 0, subY = plane ? s.subsampling_y : 0;
                if (b.m_decoded.getFlag(plane, (sbRow >> subY) - 1, (sbCol >> subX) + n4w))
                    r.ii_edge |= 1 << (2 * plane);
                if (b.m_decoded.getFlag(plane, (sbRow >> subY) + n4h, (sbCol >> subX) - 1))
                    r.ii_edge |= 2 << (2 * plane);
            }
        }
        // palette (Block::Palette, Block.cpp:2221-2298)
        if (b.PaletteSizeY || b.PaletteSizeUV) {
            auto& pal = b.m_palette;
            r.palette_off = (uint32_t)cur.palette.size();
            uint8_t hdr[AV1R_PALETTE_HDR];
            memset(hdr, 0, sizeof(hdr));
            const auto& my = pal.ColorMapY;
            const auto& muv = pal.ColorMapUV;
            hdr[0] = b.PaletteSizeY && !my.empty() ? (uint8_t)my[0].size() : 0;
            hdr[1] = b.PaletteSizeY ? (uint8_t)my.size() : 0;
            hdr[2] = b.PaletteSizeUV && !muv.empty() ? (uint8_t)muv[0].size() : 0;
            hdr[3] = b.PaletteSizeUV ? (uint8_t)muv.size() : 0;
            for (int i = 0; i < 8; i++) {
                if (i < (int)pal.palette_colors_y.size())
                    hdr[4 + i] = pal.palette_colors_y[i];
                if (i < (int)pal.palette_colors_u.size())
                    hdr[12 + i] = pal.palette_colors_u[i];
                if (i < (int)pal.palette_colors_v.size())
                    hdr[20 + i] = pal.palette_colors_v[i];
            }
            cur.palette.insert(cur.palette.end(), hdr, hdr + AV1R_PALETTE_HDR);
            if (hdr[1])
                for (auto& row : my)
                    cur.palette.insert(cur.palette.end(), row.begin(), row.end());
            if (hdr[3])
                for (auto& row : muv)
                    cur.palette.insert(cur.palette.end(), row.begin(), row.end());
            while (cur.palette.size() & 3)
                cur.palette.push_back(0);
        }
        {  // v2: the block's mode info, as stored over its 4x4 units
            const ModeInfoBlock& m = b.m_frame.m_modeInfo[b.MiRow][b.MiCol];
            for (int l = 0; l < 2; l++) {
                r.mv[l][0] = m.Mvs[l].mv[0];
                r.mv[l][1] = m.Mvs[l].mv[1];
                r.ref_frame[l] = (int8_t)m.RefFrames[l];
            }
            r.filt = (uint8_t)((m.InterpFilters[0] & 15) | (m.InterpFilters[1] << 4));
            for (int i = 0; i < 4; i++)
                r.delta_lf[i] = m.DeltaLFs[i];
        }
        r.first_tb = (uint32_t)cur.tbs.size();
        uint32_t blockIdx = (uint32_t)cur.blocks.size();
        cur.blocks.push_back(r);

        b.compute_prediction(frame, dec.m_store);

        if (b.is_inter && b.motion_mode == LOCALWARP && b.m_localWarp.LocalValid) {
            cur.blocks[blockIdx].flags |= AV1R_BLK_LOCAL_VALID;
            for (int i = 0; i < 6; i++)
                cur.blocks[blockIdx].local_warp[i] = b.m_localWarp.LocalWarpParams[i];
        }
        cur.blocks[blockIdx].flags |= f;

        // transform blocks in decode order (TransformBlock::decode, TransformBlock.cpp:2376-2456)
        for (auto& tbp : b.m_transformBlocks) {
            TransformBlock& t = *tbp;
            int plane = t.plane;
            int subX = plane ? s.subsampling_x : 0;
            int subY = plane ? s.subsampling_x : 0; // as the reference (TransformBlock.cpp:2379)
            int row = (t.y << subY) >> MI_SIZE_LOG2;
            int col = (t.x << subX) >> MI_SIZE_LOG2;
            int sbRow = row & b.sbMask, sbCol = col & b.sbMask;
            int stepX = Tx_Width[t.txSz] >> MI_SIZE_LOG2;
            int stepY = Tx_Height[t.txSz] >> MI_SIZE_LOG2;
            int maxX = (b.m_frame.MiCols * MI_SIZE) >> subX;
            int maxY = (b.m_frame.MiRows * MI_SIZE) >> subY;
            if (!(t.x >= maxX || t.y >= maxY)) {
                av1r_tb tr;
                memset(&tr, 0, sizeof(tr));
                tr.block = blockIdx;
                tr.x = t.x;
                tr.y = t.y;
                tr.plane = plane;
                tr.tx_size = t.txSz;
                tr.tx_type = t.m_eob ? t.PlaneTxType : 0;
                bool haveL = (plane == 0 ? b.AvailL : b.AvailLChroma) || t.x > t.m_baseX;
                bool haveA = (plane == 0 ? b.AvailU : b.AvailUChroma) || t.y > t.m_baseY;
                bool haveAR = b.m_decoded.getFlag(plane, (sbRow >> subY) - 1, (sbCol >> subX) + stepX);
                bool haveBL = b.m_decoded.getFlag(plane, (sbRow >> subY) + stepY, (sbCol >> subX) - 1);
                tr.flags = (haveL ? AV1R_TB_HAVE_LEFT : 0) | (haveA ? AV1R_TB_HAVE_ABOVE : 0)
                    | (haveAR ? AV1R_TB_HAVE_AR : 0) | (haveBL ? AV1R_TB_HAVE_BL : 0);
                tr.coef_off = (uint32_t)cur.coefs.size();
                if (t.m_eob) {
                    for (int i = 0; i < t.th; i++) {
                        for (int j = 0; j < t.tw; j++) {
                            int pos = i * t.tw + j;
                            int v = t.Quant[pos];
                            if (v) {
                                if (v >= (1 << 21) || v < -(1 << 21)) {
                                    fprintf(stderr, "coefficient out of packable range\n");
                                    exit(3);
                                }
                                cur.coefs.push_back(((uint32_t)v << 10) | (uint32_t)pos);
                            }
                        }
                    }
                }
                tr.coef_cnt = (uint16_t)(cur.coefs.size() - tr.coef_off);
                if (t.m_eob && !tr.coef_cnt) {
                    fprintf(stderr, "eob>0 with no non-zero coefficient\n");
                    exit(3);
                }
                if (plane && !b.is_inter) {
                    cur.blocks[blockIdx].max_luma_w = (uint16_t)b.MaxLumaW;
                    cur.blocks[blockIdx].max_luma_h = (uint16_t)b.MaxLumaH;
                }
                cur.tbs.push_back(tr);
            }
            t.decode(frame);
        }
        cur.blocks[blockIdx].n_tbs = (uint32_t)cur.tbs.size() - cur.blocks[blockIdx].first_tb;
    }

    void walk(Partition& p, std::shared_ptr<YuvFrame>& frame)
    {
        for (auto& bt : p.m_blocks) {
            if (Block* b = dynamic_cast<Block*>(bt.get()))
                dumpBlock(*b, frame);
            else if (Partition* q = dynamic_cast<Partition*>(bt.get()))
                walk(*q, frame);
        }
    }

    void fillHeader(const FrameHeader& h)
    {
        const SequenceHeader& s = *h.m_sequence;
        av1r_frame_hdr& o = cur.hdr;
        memset(&o, 0, sizeof(o));
        o.version = AV1R_VERSION;
        o.frame_width = h.FrameWidth;
        o.frame_height = h.FrameHeight;
        o.mi_cols = h.MiCols;
        o.mi_rows = h.MiRows;
        o.mi_stride = h.AlignedMiCols;
        o.mi_rows_alloc = h.AlignedMiRows;
        o.sb128 = s.use_128x128_superblock;
        o.subx = s.subsampling_x;
        o.suby = s.subsampling_y;
        o.bitdepth = s.BitDepth;
        o.show_frame = h.show_frame;
        o.show_existing_frame = h.show_existing_frame;
        o.frame_to_show = h.frame_to_show_map_idx;
        o.refresh_frame_flags = h.refresh_frame_flags;
        o.frame_type = h.frame_type;
        o.enable_intra_edge_filter = s.enable_intra_edge_filter;
        o.force_integer_mv = h.force_integer_mv;
        o.allow_intrabc = h.allow_intrabc;
        for (int i = 0; i < 8; i++)
            o.ref_frame_idx[i] = i < REFS_PER_FRAME ? h.ref_frame_idx[i] : -1;
        for (int r = 0; r < 8; r++) {
            o.gm_type[r] = h.GmType[r];
            for (int k = 0; k < 6; k++)
                o.gm_params[r][k] = h.gm_params[r][k];
            if (r >= LAST_FRAME && !h.FrameIsIntra) {
                int d = std::abs(h.get_relative_dist((uint8_t)r));
                o.ref_dist[r] = (uint8_t)CLIP3(0, MAX_FRAME_DISTANCE, d);
            }
        }
        const Quantization& q = h.m_quant;
        o.delta_q_y_dc = q.DeltaQYDc;
        o.delta_q_u_dc = q.DeltaQUDc;
        o.delta_q_u_ac = q.DeltaQUAc;
        o.delta_q_v_dc = q.DeltaQVDc;
        o.delta_q_v_ac = q.DeltaQVAc;
        const LoopFilterParams& lf = h.m_loopFilter;
        for (int i = 0; i < 4; i++)
            o.lf_level[i] = lf.loop_filter_level[i];
        o.lf_sharpness = lf.loop_filter_sharpness;
        o.lf_delta_enabled = lf.loop_filter_delta_enabled;
        o.delta_lf_multi = h.m_deltaLf.delta_lf_multi;
        for (int i = 0; i < 8; i++)
            o.lf_ref_deltas[i] = lf.loop_filter_ref_deltas[i];
        o.lf_mode_deltas[0] = lf.loop_filter_mode_deltas[0];
        o.lf_mode_deltas[1] = lf.loop_filter_mode_deltas[1];
        const CdefParams& cd = h.m_cdef;
        o.cdef_damping = cd.CdefDamping;
        o.cdef_bits = cd.cdef_bits;
        for (int i = 0; i < (1 << cd.cdef_bits); i++) {  // the rest is never written
            o.cdef_y_pri[i] = cd.cdef_y_pri_strength[i];
            o.cdef_y_sec[i] = cd.cdef_y_sec_strength[i];
            o.cdef_uv_pri[i] = cd.cdef_uv_pri_strength[i];
            o.cdef_uv_sec[i] = cd.cdef_uv_sec_strength[i];
        }
    }

    // frame-level tables known only after reconstruction (LoopfilterTxSizes) or parse.
    void fillFrameTables(const FrameHeader& h)
    {
        const SequenceHeader& s = *h.m_sequence;
        av1r_frame_hdr& o = cur.hdr;
        cur.mi.assign((size_t)h.AlignedMiRows * h.AlignedMiCols, av1r_mi());
        for (uint32_t r = 0; r < h.AlignedMiRows; r++) {
            for (uint32_t c = 0; c < h.AlignedMiCols; c++) {
                const ModeInfoBlock& m = h.m_modeInfo[r][c];
                av1r_mi& d = cur.mi[(size_t)r * h.AlignedMiCols + c];
                memset(&d, 0, sizeof(d));
                for (int l = 0; l < 2; l++) {
                    d.mv[l][0] = m.Mvs[l].mv[0];
                    d.mv[l][1] = m.Mvs[l].mv[1];
                    d.ref_frame[l] = (int8_t)m.RefFrames[l];
                }
                d.mi_size = m.MiSize;
                d.y_mode = m.YMode;
                d.uv_mode = m.UVMode;
                d.filt = (uint8_t)((m.InterpFilters[0] & 15) | (m.InterpFilters[1] << 4));
                d.flags = (m.Skip ? AV1R_MI_SKIP : 0) | (m.IsInter ? AV1R_MI_INTER : 0);
                for (int p = 0; p < 3; p++)
                    d.lf_tx[p] = m.LoopfilterTxSizes[p];
                for (int i = 0; i < 4; i++)
                    d.delta_lf[i] = m.DeltaLFs[i];
            }
        }
        o.cdef_rows = (h.MiRows + 15) / 16;
        o.cdef_cols = (h.MiCols + 15) / 16;
        cur.cdef.assign((size_t)o.cdef_rows * o.cdef_cols, -1);
        for (int r = 0; r < o.cdef_rows; r++)
            for (int c = 0; c < o.cdef_cols; c++)
                cur.cdef[(size_t)r * o.cdef_cols + c] = (int8_t)h.m_cdef.cdef_idx[r * 16][c * 16];
        const LoopRestorationpParams& lr = h.m_loopRestoration;
        o.uses_lr = lr.UsesLr;
        cur.lr.clear();
        for (int p = 0; p < 3; p++) {
            o.lr_type[p] = lr.FrameRestorationType[p];
            o.lr_unit_off[p] = (int32_t)cur.lr.size();
            if (!lr.UsesLr || lr.FrameRestorationType[p] == RESTORE_NONE)
                continue;
            int subX = p ? s.subsampling_x : 0, subY = p ? s.subsampling_y : 0;
            int us = lr.LoopRestorationSize[p];
            o.lr_unit_size[p] = us;
            int rows = std::max((ROUND2((int)h.FrameHeight, subY) + (us >> 1)) / us, 1);
            int cols = std::max((ROUND2((int)h.UpscaledWidth, subX) + (us >> 1)) / us, 1);
            o.lr_unit_rows[p] = rows;
            o.lr_unit_cols[p] = cols;
            for (int r = 0; r < rows; r++) {
                for (int c = 0; c < cols; c++) {
                    av1r_lr_unit u;
                    memset(&u, 0, sizeof(u));
                    u.type = lr.LrType[p][r][c];
                    u.sgr_set = lr.LrSgrSet[p][r][c];
                    u.sgr_xqd[0] = lr.LrSgrXqd[p][r][c][0];
                    u.sgr_xqd[1] = lr.LrSgrXqd[p][r][c][1];
                    for (int pass = 0; pass < 2; pass++)
                        for (int i = 0; i < 3; i++)
                            u.wiener[pass][i] = lr.LrWiener[p][r][c][pass][i];
                    cur.lr.push_back(u);
                }
            }
        }
    }

    void emitOutput(const std::shared_ptr<YuvFrame>& f)
    {
        for (int p = 0; p < 3; p++) {
            int w = p ? f->width >> 1 : f->width;
            int h = p ? f->height >> 1 : f->height;
            for (int y = 0; y < h; y++)
                MD5_Update(&outCtx, f->data[p] + y * f->strides[p], w);
        }
    }

    bool decodeFrame(Tiles& tiles)
    {
        FrameHeader& h = *dec.m_frame;
        const SequenceHeader& s = *h.m_sequence;
        if (s.BitDepth != 8 || !s.subsampling_x || !s.subsampling_y || h.use_superres) {
            fprintf(stderr, "unsupported stream\n");
            return false;
        }
        cur = Batch();
        fillHeader(h);
        std::shared_ptr<YuvFrame> frame = YuvFrame::create(h.FrameWidth, h.FrameHeight);
        int sbSize4 = s.use_128x128_superblock ? 32 : 16;
        for (auto& t : tiles) {
            while (!t->m_sbs.empty()) {
                std::shared_ptr<SuperBlock> sb = t->m_sbs.front();
                t->m_decoded.clear_block_decoded_flags(sb->m_r, sb->m_c, sbSize4);
                walk(*sb, frame);
                t->m_sbs.pop_front();
            }
        }
        dec.frame_end_update_cdf(tiles);
        fillFrameTables(h);
        std::string hRecon = md5_planes(*frame);
        if (const char* dir = getenv("REFDUMP_PLANES")) {
            // debug aid: raw visible planes of each stage, <dir>/f<N>_<stage>.yuv
            auto dump = [&](const YuvFrame& f, const char* tag) {
                char path[512];
                snprintf(path, sizeof(path), "%s/f%d_%s.yuv", dir, frameNo, tag);
                FILE* fp = fopen(path, "wb");
                for (int p = 0; p < 3; p++) {
                    int w = p ? f.width >> 1 : f.width, hh = p ? f.height >> 1 : f.height;
                    for (int y = 0; y < hh; y++)
                        fwrite(f.data[p] + y * f.strides[p], 1, w, fp);
                }
                fclose(fp);
            };
            dump(*frame, "recon");
        }
        const char* planeDir = getenv("REFDUMP_PLANES");
        auto dumpStage = [&](const YuvFrame& f, const char* tag) {
            if (!planeDir) return;
            char path[512];
            snprintf(path, sizeof(path), "%s/f%d_%s.yuv", planeDir, frameNo, tag);
            FILE* fp = fopen(path, "wb");
            for (int p = 0; p < 3; p++) {
                int w = p ? f.width >> 1 : f.width, hh = p ? f.height >> 1 : f.height;
                for (int y = 0; y < hh; y++) fwrite(f.data[p] + y * f.strides[p], 1, w, fp);
            }
            fclose(fp);
        };
        LoopFilter lf(dec.m_frame);
        lf.filter(frame);
        std::string hLf = md5_planes(*frame);
        dumpStage(*frame, "lf");
        Cdef cdef(dec.m_frame);
        std::shared_ptr<YuvFrame> cdefFrame = cdef.filter(frame);
        std::string hCdef = md5_planes(*cdefFrame);
        dumpStage(*cdefFrame, "cdef");
        std::shared_ptr<YuvFrame> upCdef = dec.upscaling(cdefFrame);
        std::shared_ptr<YuvFrame> upCur = dec.upscaling(frame);
        LoopRestoration lr(dec.m_frame, upCdef, upCur);
        std::shared_ptr<YuvFrame> lrFrame = lr.filter();
        std::string hLr = md5_planes(*lrFrame);
        dumpStage(*lrFrame, "lr");
        dec.m_frame->motionVectorStorage();
        write_batch(out, cur);
        fprintf(hashes, "%d %d %d %d %s %s %s %s %zu %zu %zu\n", frameNo, (int)h.frame_type,
            (int)h.show_frame, 0, hRecon.c_str(), hLf.c_str(), hCdef.c_str(), hLr.c_str(),
            cur.blocks.size(), cur.tbs.size(), cur.coefs.size());
        frameNo++;
        if (h.show_frame)
            emitOutput(lrFrame);
        dec.updateFrameStore(h, lrFrame);
        dec.m_parser->finishFrame();
        return true;
    }

    void showExisting()
    {
        FrameHeader& h = *dec.m_frame;
        cur = Batch();
        fillHeader(h);
        write_batch(out, cur);
        const std::shared_ptr<YuvFrame>& f = dec.m_store[h.frame_to_show_map_idx];
        std::string hf = md5_planes(*f);
        fprintf(hashes, "%d %d %d %d %s %s %s %s 0 0 0\n", frameNo, (int)h.frame_type, 1, 1,
            hf.c_str(), hf.c_str(), hf.c_str(), hf.c_str());
        frameNo++;
        emitOutput(f);
        dec.updateFrameStore(h, f);
        h.referenceFrameLoading();
        h.motionVectorStorage();
        dec.m_parser->finishFrame();
    }

    // mirrors Decoder::decode (Av1Decoder.cpp:49-109)
    bool decodeTemporalUnit(uint8_t* data, size_t size)
    {
        BitReader reader(data, size);
        while (reader.getRemainingBitsCount() > 0) {
            obu_header header;
            if (!header.parse(reader))
                return false;
            bool ret = true;
            ObuType type = header.obu_type;
            uint64_t sz = header.obu_size;
            BitReader br(data + (reader.getPos() >> 3), sz);
            Parser& parser = *dec.m_parser;
            if (type == OBU_SEQUENCE_HEADER) {
                ret = parser.parseSequenceHeader(br);
            } else if (type == OBU_TD) {
                ret = parser.parseTemporalDelimiter(br);
            } else if (type == OBU_FRAME_HEADER) {
                dec.m_frame = parser.parseFrameHeader(br);
                ret = bool(dec.m_frame);
                if (ret && dec.m_frame->show_existing_frame)
                    showExisting();
            } else if (type == OBU_TILE_GROUP) {
                TileGroup group;
                ret = parser.parseTileGroup(br, dec.m_frame, group);
                if (ret) {
                    dec.m_tiles.insert(dec.m_tiles.end(), group.begin(), group.end());
                    if (dec.m_tiles.size() == parser.m_frame->NumTiles) {
                        ret = decodeFrame(dec.m_tiles);
                        dec.m_tiles.clear();
                    }
                }
            } else if (type == OBU_METADATA) {
                ret = parser.parseMetadata(br);
            } else if (type == OBU_PADDING) {
                ret = parser.parsePadding(br);
            } else if (type == OBU_FRAME) {
                TileGroup group;
                dec.m_frame = parser.parseFrame(br, group);
                ret = dec.m_frame ? decodeFrame(group) : false;
                dec.m_tiles.clear();
            }
            if (!ret)
                return false;
            reader.skip(sz << 3);
        }
        return true;
    }
};

} // namespace

int main(int argc, char** argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s in.ivf out.av1b out.hashes\n", argv[0]);
        return 1;
    }
    FILE* in = fopen(argv[1], "rb");
    if (!in) {
        perror(argv[1]);
        return 1;
    }
    std::vector<uint8_t> file;
    {
        uint8_t buf[65536];
        size_t n;
        while ((n = fread(buf, 1, sizeof(buf), in)) > 0)
            file.insert(file.end(), buf, buf + n);
        fclose(in);
    }
    if (file.size() < 32 || memcmp(file.data(), "DKIF", 4)) {
        fprintf(stderr, "not an IVF file\n");
        return 1;
    }
    Dumper d;
    d.out = fopen(argv[2], "wb");
    d.hashes = fopen(argv[3], "w");
    if (!d.out || !d.hashes)
        return 1;
    uint32_t magic = 0x42315641; // "AV1B"
    uint32_t ver = AV1R_VERSION;
    fwrite(&magic, 4, 1, d.out);
    fwrite(&ver, 4, 1, d.out);
    MD5_Init(&d.outCtx);
    size_t pos = 32;
    while (pos + 12 <= file.size()) {
        uint32_t sz = file[pos] | (file[pos + 1] << 8) | (file[pos + 2] << 16) | ((uint32_t)file[pos + 3] << 24);
        pos += 12;
        if (pos + sz > file.size())
            break;
        std::vector<uint8_t> tu(file.begin() + pos, file.begin() + pos + sz);
        pos += sz;
        if (!d.decodeTemporalUnit(tu.data(), tu.size())) {
            fprintf(stderr, "decode failed\n");
            return 2;
        }
    }
    unsigned char dg[16];
    MD5_Final(dg, &d.outCtx);
    fprintf(d.hashes, "md5 ");
    for (int i = 0; i < 16; i++)
        fprintf(d.hashes, "%02x", dg[i]);
    fprintf(d.hashes, "\n");
    fclose(d.out);
    fclose(d.hashes);
    return 0;
}
