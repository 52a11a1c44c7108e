/*
 * av1r.h -- C-ABI of the MI355X (gfx950) AV1 block-reconstruction backend.
 *
 * The boundary sits where the reference decoder (oddstone/av1dec) hands a parsed
 * frame to reconstruction: `Decoder::decodeFrame` (decoder/Av1Decoder.cpp:128-156)
 * walks every Tile's parsed SuperBlock->Partition->Block->TransformBlock tree with
 * `decode()` and then runs `decode_frame_wrapup` (Av1Decoder.cpp:171-192:
 * LoopFilter -> Cdef -> LoopRestoration).  Everything ABOVE that line (OBU/header
 * parse, od_ec entropy decoding, mode-info and coefficient parse) stays on the host;
 * everything BELOW it is this library.  The host ships one "frame batch": the frame
 * header, the per-4x4 mode-info grid, the coded blocks and transform blocks in decode
 * order, the non-zero quantized coefficients, palette maps, CDEF indices and loop
 * restoration unit parameters.  All structs are POD, little-endian, no padding holes
 * (sizes: av1r_sizeof(); checked against the Python mirror in tests/test_abi.py).
 *
 * Enumerations (BLOCK_SIZE, TX_SIZE, TX_TYPE, PREDICTION_MODE, ...) use the numeric
 * values of the reference's aom/enums.h so a reference-side binding is a field copy.
 *
 * Entry points replace (reference file:line):
 *   av1r_create / av1r_destroy        -- Decoder::Decoder / ~Decoder (Av1Decoder.cpp:40-47)
 *   av1r_decode_frame                 -- Decoder::decodeFrame + decode_frame_wrapup
 *                                        (Av1Decoder.cpp:128-156, 171-192)
 *   av1r_frame_begin/submit_tile/end  -- the same, split per Tile (Tile::decode, Tile.cpp:168-178)
 *   av1r_show_existing                -- Decoder::showExistingFrame (Av1Decoder.cpp:158-169)
 *   av1r_ref_release                  -- a slot dropped from the FrameStore (updateFrameStore,
 *                                        Av1Decoder.cpp:111-119)
 *   av1r_output_pending/av1r_get_output -- Decoder::getOutput (Av1Decoder.cpp:203-211) +
 *                                        the I420 row copy of DecodeOutput::output
 *                                        (tests/DecodeOutput.cpp:48-69)
 *   av1r_get_output_async / av1r_output_query / av1r_output_wait
 *                                     -- the same read-back overlapped with later frames' decoding
 *   av1r_read_stage                   -- debug read-back of one pipeline stage
 *                                        (the reference's DUMP hooks, Av1Decoder.cpp:142-152)
 */
#ifndef AV1R_H
#define AV1R_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AV1R_VERSION 2u

/* ---- status codes (map onto YamiStatus, interface/VideoCommonDefs.h:130-164) ---- */
#define AV1R_OK 0
#define AV1R_E_INVALID (-1)      /* malformed batch / bad argument  (YAMI_INVALID_PARAM) */
#define AV1R_E_UNSUPPORTED (-2)  /* feature outside the reference's support (YAMI_UNSUPPORTED) */
#define AV1R_E_DEVICE (-3)       /* HIP error (YAMI_FAIL) */
#define AV1R_E_NOMEM (-4)        /* allocation failure (YAMI_OUT_MEMORY) */
#define AV1R_E_NO_OUTPUT (-5)    /* output queue empty (getOutput() == nullptr) */

/* ---- per-4x4 mode-info record: the subset of ModeInfoBlock (decoder/Parser.h:432-455)
 *      read by reconstruction and the loop filters.  One per 4x4 of the SB-aligned grid
 *      (AlignedMiRows x AlignedMiCols, Parser.cpp:551).  24 bytes. ---- */
typedef struct av1r_mi {
    int16_t mv[2][2];     /* Mvs[refList].mv[{0=row,1=col}] in 1/8 pel            */
    int8_t ref_frame[2];  /* RefFrames[]: -1 NONE, 0 INTRA, 1..7 LAST..ALTREF       */
    uint8_t mi_size;      /* MiSize (BLOCK_SIZE)                                    */
    uint8_t y_mode;       /* YMode (PREDICTION_MODE)                                */
    uint8_t filt;         /* InterpFilters[0] | InterpFilters[1] << 4               */
    uint8_t flags;        /* AV1R_MI_SKIP | AV1R_MI_INTER                           */
    uint8_t lf_tx[3];     /* LoopfilterTxSizes[plane] (TX_SIZE)                     */
    int8_t delta_lf[4];   /* DeltaLFs[]                                             */
    uint8_t uv_mode;      /* UVMode                                                 */
    uint8_t pad[2];
} av1r_mi;
#define AV1R_MI_SKIP 1u
#define AV1R_MI_INTER 2u

/* ---- coded block (Block, decoder/Block.h:52-291).  One per Block in decode order. ---- */
typedef struct av1r_block {
    uint16_t mi_row, mi_col;
    uint8_t mi_size;           /* BLOCK_SIZE                                         */
    uint8_t qindex;            /* get_qindex(CurrentQIndex, segment_id) (Parser.cpp:1654) */
    uint8_t y_mode, uv_mode;
    int8_t angle_delta_y, angle_delta_uv;
    uint8_t filter_intra_mode; /* FILTER_INTRA_MODE, valid when AV1R_BLK_FILTER_INTRA   */
    int8_t cfl_alpha_u, cfl_alpha_v;
    uint8_t palette_size_y, palette_size_uv;
    uint8_t motion_mode;       /* SIMPLE_TRANSLATION / OBMC_CAUSAL / LOCALWARP        */
    uint8_t compound_type;     /* COMPOUND_WEDGE .. COMPOUND_DISTANCE (aom/enums.h:474) */
    uint8_t interintra_mode;   /* II_*                                               */
    uint8_t wedge_index, wedge_sign;
    uint8_t mask_type;
    uint8_t ii_edge;           /* interintra block-level haveAboveRight(bit 2p) / haveBelowLeft(bit 2p+1) */
    uint8_t pad0[2];
    uint32_t flags;            /* AV1R_BLK_*                                          */
    uint16_t max_luma_w, max_luma_h; /* MaxLumaW/H at chroma time (TransformBlock.cpp:2418-2421) */
    int32_t local_warp[6];     /* LocalWarpParams (Block.cpp:1116-1169) when AV1R_BLK_LOCAL_VALID */
    uint32_t palette_off;      /* byte offset of this block's av1r_palette record     */
    uint32_t first_tb, n_tbs;  /* this block's transform blocks in the tb array       */
    /* the block's own mode-info values (ModeInfoBlock, Parser.h:432-455; v2): with the
     * fields above and the transform blocks they determine the whole mode-info grid, which
     * the library derives on the device instead of uploading it (see av1r_frame_batch.mi) */
    int16_t mv[2][2];          /* Mvs[refList] (inter blocks; [1] zero unless compound)  */
    int8_t ref_frame[2];       /* RefFrame[] (intra: 0, -1; inter-intra: ref, 0)         */
    uint8_t filt;              /* InterpFilters[0] | InterpFilters[1] << 4 (inter only)  */
    uint8_t pad1;
    int8_t delta_lf[4];        /* DeltaLF[] at the block                                 */
} av1r_block;
#define AV1R_BLK_INTER (1u << 0)
#define AV1R_BLK_INTRABC (1u << 1)
#define AV1R_BLK_LOSSLESS (1u << 2)
#define AV1R_BLK_HAS_CHROMA (1u << 3)
#define AV1R_BLK_FILTER_INTRA (1u << 4)
#define AV1R_BLK_INTERINTRA (1u << 5)
#define AV1R_BLK_WEDGE_II (1u << 6)
#define AV1R_BLK_LOCAL_VALID (1u << 7)
#define AV1R_BLK_AVAIL_L (1u << 8)
#define AV1R_BLK_AVAIL_U (1u << 9)
#define AV1R_BLK_AVAIL_L_UV (1u << 10)
#define AV1R_BLK_AVAIL_U_UV (1u << 11)
#define AV1R_BLK_SMOOTH_A_Y (1u << 12) /* getAboveSmooth() luma  (IntraPredict.cpp:232) */
#define AV1R_BLK_SMOOTH_L_Y (1u << 13) /* getLeftSmooth()  luma  (IntraPredict.cpp:214) */
#define AV1R_BLK_SMOOTH_A_UV (1u << 14)
#define AV1R_BLK_SMOOTH_L_UV (1u << 15)
#define AV1R_BLK_SKIP (1u << 16)

/* ---- transform block (TransformBlock, decoder/TransformBlock.h:46-129). 20 bytes. ---- */
typedef struct av1r_tb {
    uint32_t block;     /* index of the owning av1r_block                              */
    uint32_t coef_off;  /* first coefficient in the coefficient stream                 */
    uint16_t x, y;      /* top-left in plane pixels (startX/startY)                    */
    uint16_t coef_cnt;  /* number of non-zero coefficients (0 <=> eob == 0)            */
    uint8_t plane;
    uint8_t tx_size;    /* TX_SIZE                                                     */
    uint8_t tx_type;    /* PlaneTxType (TX_TYPE), flips implied (TransformBlock.cpp:1658-1675) */
    uint8_t flags;      /* AV1R_TB_*                                                   */
    uint8_t pad[2];
} av1r_tb;
#define AV1R_TB_HAVE_LEFT 1u   /* predict_intra haveLeft  (TransformBlock.cpp:2411)   */
#define AV1R_TB_HAVE_ABOVE 2u  /* predict_intra haveAbove (TransformBlock.cpp:2412)   */
#define AV1R_TB_HAVE_AR 4u     /* haveAboveRight          (TransformBlock.cpp:2406)   */
#define AV1R_TB_HAVE_BL 8u     /* haveBelowLeft           (TransformBlock.cpp:2407)   */

/* Coefficient stream: one uint32 per non-zero quantized coefficient of a TB,
 * (level << 10) | pos, pos = i * min(w,32) + j (Quant[] layout, TransformBlock.cpp:2266),
 * level = signed Quant value (|level| < 2^21). */
#define AV1R_COEF_POS(c) ((int)((c) & 1023u))
#define AV1R_COEF_LEVEL(c) (((int32_t)(c)) >> 10)

/* Palette record, at av1r_block.palette_off in the palette blob:
 *   uint8 wy, hy, wuv, huv; uint8 colors[3][8];  uint8 map_y[hy*wy]; uint8 map_uv[huv*wuv]
 * (Block::Palette, Block.cpp:2221-2298; maps already border-extended). */
#define AV1R_PALETTE_HDR 28

/* ---- loop restoration unit (LrType/LrWiener/LrSgrSet/LrSgrXqd, Parser.h:384-402). 12 B ---- */
typedef struct av1r_lr_unit {
    uint8_t type;       /* RESTORE_NONE / RESTORE_WIENER / RESTORE_SGRPROJ          */
    uint8_t sgr_set;
    int8_t sgr_xqd[2];
    int8_t wiener[2][3]; /* [0] vertical, [1] horizontal (LoopRestoration.cpp:250-251) */
    uint8_t pad[2];
} av1r_lr_unit;

/* ---- frame header: what reconstruction and the filters read from FrameHeader /
 *      SequenceHeader (decoder/Parser.h:258-640). ---- */
typedef struct av1r_frame_hdr {
    uint32_t version;            /* AV1R_VERSION                                    */
    int32_t frame_width, frame_height; /* FrameWidth / FrameHeight (no superres)    */
    int32_t mi_cols, mi_rows;    /* MiCols / MiRows                                 */
    int32_t mi_stride, mi_rows_alloc; /* AlignedMiCols / AlignedMiRows (mi grid dims) */
    uint8_t sb128, subx, suby, bitdepth;
    uint8_t show_frame, show_existing_frame, frame_to_show, refresh_frame_flags;
    uint8_t frame_type, enable_intra_edge_filter, force_integer_mv, allow_intrabc;
    int8_t ref_frame_idx[8];     /* ref_frame_idx[ref - LAST_FRAME] (7 used)         */
    uint8_t gm_type[8];          /* GmType[ref]                                     */
    int32_t gm_params[8][6];     /* gm_params[ref][]                                */
    uint8_t ref_dist[8];         /* Clip3(0, MAX_FRAME_DISTANCE, |get_relative_dist(ref)|) */
    int8_t delta_q_y_dc, delta_q_u_dc, delta_q_u_ac, delta_q_v_dc, delta_q_v_ac;
    /* loop filter (LoopFilterParams, DeltaLf) */
    uint8_t lf_level[4], lf_sharpness, lf_delta_enabled, delta_lf_multi;
    int8_t lf_ref_deltas[8], lf_mode_deltas[2];
    /* CDEF (CdefParams) */
    uint8_t cdef_damping, cdef_bits;
    uint8_t cdef_y_pri[8], cdef_y_sec[8], cdef_uv_pri[8], cdef_uv_sec[8];
    int32_t cdef_rows, cdef_cols;  /* cdef_idx grid dims (64x64 units)               */
    /* loop restoration */
    uint8_t uses_lr, lr_type[3];   /* UsesLr, FrameRestorationType[]                 */
    int32_t lr_unit_size[3];
    int32_t lr_unit_rows[3], lr_unit_cols[3];
    int32_t lr_unit_off[3];        /* first unit of each plane in the lr unit array  */
    uint8_t reserved[16];
} av1r_frame_hdr;

/* ---- one frame's (or one tile's) payload ---- */
typedef struct av1r_frame_batch {
    const av1r_frame_hdr* hdr;
    /* mi_rows_alloc * mi_stride records, or NULL.  The grid is a function of the blocks
     * (their mode info over their 4x4 units) and transform blocks (lf_tx over the units each
     * covers, TransformBlock.cpp:2444-2454), zero elsewhere: the library derives it on the
     * device (k_mi) and never reads this array -- host consumers (the CPU oracle) may. */
    const av1r_mi* mi;
    const av1r_block* blocks;
    uint32_t n_blocks;
    const av1r_tb* tbs;
    uint32_t n_tbs;
    const uint32_t* coefs;
    uint32_t n_coefs;
    const uint8_t* palette;
    uint32_t n_palette;            /* bytes                                           */
    const int8_t* cdef_idx;        /* cdef_rows * cdef_cols, -1 = off                 */
    const av1r_lr_unit* lr_units;
    uint32_t n_lr_units;
} av1r_frame_batch;

typedef struct av1r_ctx av1r_ctx;

/* Stage ids for av1r_read_stage. */
#define AV1R_STAGE_RECON 0
#define AV1R_STAGE_LF 1
#define AV1R_STAGE_CDEF 2
#define AV1R_STAGE_LR 3

/* Create a decoding context bound to HIP device `device` and its own HIP stream. */
int av1r_create(int device, av1r_ctx** out);
void av1r_destroy(av1r_ctx* ctx);

/* Decode (reconstruct + filter) one frame and update the reference store. */
int av1r_decode_frame(av1r_ctx* ctx, const av1r_frame_batch* batch);

/* Split form of av1r_decode_frame: header-level data first, then each tile's blocks
 * (blocks/tbs/coefs/palette fields of the batch; block indices and offsets are local to
 * the tile), then frame_end runs recon -> LF -> CDEF -> LR. */
int av1r_frame_begin(av1r_ctx* ctx, const av1r_frame_batch* frame_level);
int av1r_submit_tile(av1r_ctx* ctx, const av1r_frame_batch* tile);
int av1r_frame_end(av1r_ctx* ctx);

/* Device-resident frames: validate, schedule and upload a batch once (outside any
 * timed region), then decode it from HBM.  Handles stay valid until released. */
int av1r_prepare(av1r_ctx* ctx, const av1r_frame_batch* batch, int* handle);
int av1r_decode_prepared(av1r_ctx* ctx, int handle);
/* Batched form over n independent streams: frame handles[i] of context
 * ctxs[i] (all on one device, each context at most once) go through recon -> LF -> CDEF
 * -> LR in shared launches on ctxs[0]'s stream -- every stream's dependency level in one
 * k_level launch, every stream's frame in one launch per filter.  Same results as n
 * av1r_decode_prepared calls. */
int av1r_decode_prepared_batch(av1r_ctx* const* ctxs, const int* handles, int n);
int av1r_release_prepared(av1r_ctx* ctx, int handle);

/* Host-pipelined decoding (the parse -> schedule -> GPU pipeline of SURVEY.md 8f rank 4).
 * av1r_pack validates, schedules and packs one frame batch into pinned host memory: it
 * needs no context and is thread-safe, so worker threads pack frames t+1, t+2, ... while
 * the GPU decodes frame t.  av1r_decode_packed_batch uploads each packed frame (async, on
 * the lead context's copy stream, overlapping the previous batch's kernels) and decodes
 * frame i of context ctxs[i] in shared launches, as av1r_decode_prepared_batch.  A packed
 * frame may be freed (returned to the library's pool) as soon as the call returns;
 * av1r_pack_last_error describes the calling thread's last av1r_pack failure. */
typedef struct av1r_packed av1r_packed;
int av1r_pack(const av1r_frame_batch* batch, av1r_packed** out);
void av1r_packed_free(av1r_packed* p);
size_t av1r_packed_bytes(const av1r_packed* p);
/* The packed frame's host bytes that travel to the device (*bytes: their count): for
 * inspection and tests (e.g. that packing is deterministic). */
const void* av1r_packed_data(const av1r_packed* p, size_t* bytes);
const char* av1r_pack_last_error(void);
int av1r_decode_packed_batch(av1r_ctx* const* ctxs, av1r_packed* const* frames, int n);
/* Profiling hook (environment AV1R_PACK_PROF=1): ns[0..5] = nanoseconds all threads spent
 * in av1r_pack's phases (validation, schedule set-up, per-block dependencies, item lists,
 * dependency lists, packing copy), ns[6] = frames packed; returns the phase count (6), or 0
 * when profiling is off.  reset = 1 zeroes the counters afterwards. */
int av1r_pack_profile(uint64_t* ns, int n, int reset);
/* In both batched entry points a frame with a deep dependency chain (a key frame) is
 * launched alone on its own context's stream, overlapping the batch.  av1r_busy returns 1
 * while such a frame is still running: a scheduler leaves that stream out of the next
 * batches until then, so they never wait for the chain. */
int av1r_busy(av1r_ctx* ctx);
/* Do not queue shown frames for read-back (they still refresh the reference store). */
int av1r_set_discard_output(av1r_ctx* ctx, int discard);

/* show_existing_frame: queue slot `slot` for output and refresh per `refresh_flags`. */
int av1r_show_existing(av1r_ctx* ctx, int slot, int refresh_flags);
/* Drop the reference store's hold on the slots in `slot_mask` (bit i = slot i), as the
 * reference drops a slot's shared_ptr when updateFrameStore replaces it
 * (Av1Decoder.cpp:111-119) -- for a caller that resets or flushes a stream between GOPs.
 * Refresh releases the replaced frames by itself, so a decoder running a stream never needs
 * it.  Work already queued that reads those slots completes first (the frames are
 * refcounted); a later frame that references an emptied slot fails validation with
 * AV1R_E_INVALID. */
int av1r_ref_release(av1r_ctx* ctx, int slot_mask);

/* Output queue.  av1r_get_output copies the oldest queued frame's visible I420 planes
 * (width x height, (width>>1) x (height>>1)) into the caller's buffers and pops it. */
int av1r_output_pending(av1r_ctx* ctx);
int av1r_get_output(av1r_ctx* ctx, uint8_t* y, int y_stride, uint8_t* u, int u_stride,
                    uint8_t* v, int v_stride, int* width, int* height);

/* Asynchronous form (the same Decoder::getOutput, Av1Decoder.cpp:203-211, without the
 * wait): pops the oldest queued frame and returns at once with a ticket.  The frame's
 * visible I420 planes are copied into the caller's buffers on the context's own read-back
 * stream as soon as its kernels have completed, so the copy overlaps the decoding of later
 * frames; the buffers must stay valid until the ticket is waited for, and should be pinned
 * (hipHostMalloc) for the copy to be a DMA.  av1r_output_query advances a ticket without
 * blocking (1: the bytes have landed, 0: not yet; it issues the copy once the frame is
 * done); av1r_output_start only issues the copy if the frame is done (1: issued now or
 * before, 0: the frame is still decoding) -- a driver holding several tickets starts every
 * finished frame's copy at once; av1r_output_wait blocks until they have landed, releases
 * the ticket (and the frame), and returns AV1R_E_DEVICE for a frame a device error touched.
 * A ticket belongs to the context's driving thread; av1r_destroy releases tickets never
 * waited for. */
typedef struct av1r_output_ticket av1r_output_ticket;
int av1r_get_output_async(av1r_ctx* ctx, uint8_t* y, int y_stride, uint8_t* u, int u_stride,
                          uint8_t* v, int v_stride, int* width, int* height, av1r_output_ticket** ticket);
int av1r_output_query(av1r_output_ticket* ticket);
int av1r_output_start(av1r_output_ticket* ticket);
int av1r_output_wait(av1r_output_ticket* ticket);
/* 1: from now on every shown frame's read-back starts as soon as it is queued (into pinned
 * staging memory of the context, on its read-back stream), so av1r_get_output waits for
 * that copy alone -- the blocking getOutput of the Yami / YamiAv1 facades overlapping the
 * decoding of the next frames.  (av1r_get_output_async is refused while frames are staged.) */
int av1r_set_output_prefetch(av1r_ctx* ctx, int on);

/* Copy the visible region of plane `plane` of stage `stage` of the last decoded frame. */
int av1r_read_stage(av1r_ctx* ctx, int stage, int plane, uint8_t* dst, int dst_stride);

/* Timing / profiling helpers (bench). */
int av1r_synchronize(av1r_ctx* ctx);
/* Average device time (ms) of the last frame's kernels, by class; filled by the bench. */
int av1r_last_frame_times(av1r_ctx* ctx, float* recon_ms, float* lf_ms, float* cdef_ms,
                          float* lr_ms);
int av1r_set_timing(av1r_ctx* ctx, int enable);
/* With timing on: synchronise, return the summed device time (ms) of the recon / LF /
 * CDEF / LR stages of every frame launched since the previous call, and reset. */
int av1r_stage_times(av1r_ctx* ctx, float* totals4, int* frames);
/* With timing on: the recon stage of the same frames split by kernel -- k_inter, k_resid
 * (both residual launches), k_flow (incl. its stream hand-off) -- in k_flow mode; call
 * BEFORE av1r_stage_times (which resets the record). */
int av1r_recon_kernel_times(av1r_ctx* ctx, float* totals3, int* frames);
/* Reconstruction schedule of the frames this context launches (a batch follows its first
 * context): 1 = the dataflow kernel k_flow (default; frames with intra block copy still
 * use level launches), 0 = one launch per dependency level, -1 = the default (environment
 * AV1R_FLOW=0 selects level launches).  Both are bit-exact; level launches are slower. */
int av1r_set_schedule(av1r_ctx* ctx, int mode);
/* Keep per-stage snapshots for av1r_read_stage (default on; costs 2 frame copies). */
int av1r_set_keep_stages(av1r_ctx* ctx, int keep);
/* Dependency levels (recon launches) and uploaded batch bytes of the last frame. */
int av1r_last_frame_stats(av1r_ctx* ctx, int* levels, uint64_t* upload_bytes);
const char* av1r_last_error(av1r_ctx* ctx);
/* Test / diagnosis hooks.  av1r_set_flow_spins: polls after which a k_flow wait of this
 * context's launches gives up (0 = the default bound); 1 forces the timeout path, whose
 * frames must then surface as AV1R_E_DEVICE from av1r_get_output / av1r_synchronize.
 * av1r_flow_debug: in a -DAV1R_FLOW_DEBUG build, the number of k_flow workgroup entries
 * that found another launch's k_flow still running, the first n recorded pairs
 * (earlier epoch slot << 16 | entering epoch) and how many of those pairs were launched
 * from different streams; -1 in a normal build. */
int av1r_set_flow_spins(av1r_ctx* ctx, uint32_t spins);
int av1r_flow_debug(uint32_t* pairs, int n, int reset, int* cross_stream);
/* Process-wide: 1 = small intra transform blocks of the dataflow kernels take the lean path
 * (default; environment AV1R_FI), 0 = the generic one.  Both are bit-exact (A/B).  Returns
 * the previous value. */
int av1r_set_fast_intra(int on);
/* Removed in round 5 (the strip schedule k_strip, the fused filter kernel k_post and per-wave
 * k_flow items, each measured slower: DESIGN.md 3.1b, 4.1): kept as no-ops returning 0 for
 * one release so that existing callers still link.  Deprecated. */
int av1r_set_strip_levels(int levels);
int av1r_set_filter_fusion(int on);
int av1r_set_flow_wave(int on);
/* Host-only check of a batch: validation + dependency schedule, no device needed.
 * Returns the status; *levels = recon launch levels.  err receives the message. */
int av1r_check_batch(const av1r_frame_batch* batch, int* levels, char* err, int err_len);
/* sizeof of the ABI structs: 0 hdr, 1 mi, 2 block, 3 tb, 4 lr_unit, 5 frame_batch. */
size_t av1r_sizeof(int which);

/* ---- multi-stream pipeline (av1r_pipeline.cpp; SURVEY.md 8e + 8f rank 4) ----
 * n independent streams (contexts on one device) decoded end to end in native threads:
 * `workers` threads pull each stream's frames in decode order from `src` and pack them
 * (av1r_pack) up to `depth` ahead per stream (<= 0: max(8, 2 * ceil(workers / n))); the calling
 * thread launches one frame of every ready
 * stream per shared launch (av1r_decode_packed_batch), applies show-existing frames in
 * order (av1r_show_existing), and finally synchronizes every context.  Stops after
 * max_frames frames per stream (<= 0: at each source's end).  The reference's per-stream
 * Decoder::decode loop (decoder/Av1Decoder.cpp:49-109), reconstruction batched across
 * streams. */
typedef struct av1r_stream_source {
    /* Frame k of stream `stream` (k = 0, 1, ... per stream, only ever called from that
     * stream's producer): *batch stays valid until the next call for the same stream.
     * Returns 0 (a frame), 1 (end of stream) or a negative status. */
    int (*next)(void* user, int stream, const av1r_frame_batch** batch);
    void* user;
    /* 1: a returned batch stays valid until the run ends (then several frames of a stream
     * are packed concurrently); 0: only until the next call for that stream; 2: until the
     * pipeline hands it back through `release` (called once per batch `next` returned, when
     * it has been packed), so the next frame's fetch overlaps this one's packing */
    int stable;
    void (*release)(void* user, int stream, const av1r_frame_batch* batch);  /* stable == 2 only */
} av1r_stream_source;
typedef struct av1r_pipeline_stats {
    uint64_t frames;   /* frames decoded (shown-existing included), all streams          */
    uint64_t batches;  /* shared launches                                                  */
    double elapsed_s;  /* wall time of the run, synchronisation included                  */
    double produce_s;  /* producer time in src->next (e.g. parsing), summed over streams  */
    double pack_s;     /* producer time in av1r_pack, summed over streams                 */
    double wait_s;     /* launcher time with no stream ready                               */
    double launch_s;   /* launcher time inside av1r_decode_packed_batch                    */
    double output_s;   /* launcher time delivering frames (av1r_pipeline_set_output)       */
} av1r_pipeline_stats;
int av1r_pipeline_run(av1r_ctx* const* ctxs, int n, const av1r_stream_source* src, int64_t max_frames, int depth,
                      int workers, av1r_pipeline_stats* stats);
/* The same pipeline kept open between runs: av1r_pipeline_open starts the workers, which
 * from then on keep every stream `depth` frames ahead (no frame budget: a cycling source
 * is fetched for as long as the pipeline is open); each av1r_pipeline_step launches
 * `frames` more entries of every stream (frames and show-existing units; 0: to every
 * stream's end) and returns once every context is synchronized -- so consecutive steps see
 * the steady state of a decoder that never stops (av1r_pipeline_run = open + one step +
 * close, with the workers stopping at max_frames).  av1r_pipeline_launched: the entries
 * launched per stream so far (counts[n], n = the pipeline's stream count).
 * av1r_pipeline_close stops the workers and frees what they packed ahead. */
typedef struct av1r_pipeline av1r_pipeline;
int av1r_pipeline_open(av1r_ctx* const* ctxs, int n, const av1r_stream_source* src, int depth, int workers,
                       av1r_pipeline** out);
int av1r_pipeline_step(av1r_pipeline* p, int64_t frames, av1r_pipeline_stats* stats);
int av1r_pipeline_launched(const av1r_pipeline* p, int64_t* counts, int n);
void av1r_pipeline_close(av1r_pipeline* p);
/* Frame delivery from a pipeline (the reference application's getOutput after every
 * decode call, tests/Av1Dec.cpp:216-220): with a sink set, the launching thread starts the
 * read-back of every shown frame as soon as it is launched (av1r_get_output_async into the
 * buffer `acquire` gives: planes[3] / strides[3] for a width x height I420 frame of
 * `stream`; nonzero = error, the step fails), keeps decoding, and calls `deliver` for each
 * frame once its bytes have landed, in order per stream (status AV1R_OK or AV1R_E_DEVICE).
 * At most AV1R_SINK_INFLIGHT read-backs per stream are outstanding, so a sink needs that
 * many buffers per stream in rotation; every frame of a step is delivered before the step
 * returns.  NULL: shown frames stay queued in their contexts (av1r_get_output). */
#define AV1R_SINK_INFLIGHT 8
typedef struct av1r_output_sink {
    int (*acquire)(void* user, int stream, int width, int height, uint8_t** planes, int* strides);
    void (*deliver)(void* user, int stream, int status);
    void* user;
} av1r_output_sink;
int av1r_pipeline_set_output(av1r_pipeline* p, const av1r_output_sink* sink);
/* The library's frame layout in device memory: plane p of a width x height frame starts
 * offsets[p] bytes after plane 0, rows strides[p] apart; `span` = plane 0's first byte to
 * the last visible byte of plane 2.  A read-back destination laid out the same way (planes
 * at those offsets from planes[0], those strides) travels as ONE linear copy of `span`
 * bytes instead of three 2-D copies. */
int av1r_frame_layout(int width, int height, int* strides, size_t* offsets, size_t* span);
/* A sink of pinned host buffers (hipHostMalloc): `slots` (>= AV1R_SINK_INFLIGHT) frames of
 * at most width x height per stream in the av1r_frame_layout of each frame, reused in
 * rotation; it counts what it was delivered (av1r_ring_sink_delivered: frames of `stream`,
 * -1 for a bad argument) and a frame's buffer is readable from its delivery until `slots`
 * later frames of that stream have been acquired (av1r_ring_sink_frame: plane 0 of the
 * stream's k-th delivered frame, the others at the layout's offsets; NULL once
 * overwritten). */
int av1r_ring_sink_create(int n_streams, int width, int height, int slots, av1r_output_sink* out);
void av1r_ring_sink_destroy(av1r_output_sink* sink);
int64_t av1r_ring_sink_delivered(const av1r_output_sink* sink, int stream);
const uint8_t* av1r_ring_sink_frame(const av1r_output_sink* sink, int stream, int64_t k, int* width, int* height);
/* Source over in-memory batches: stream s (< n_streams) yields batches[s][pos[s] % count[s]],
 * then advances pos[s] (use av1r_cycle_next as `next` and an av1r_cycle as `user`).  It
 * never ends, so av1r_pipeline_run rejects it (AV1R_E_INVALID) without max_frames > 0 or
 * with fewer than n streams. */
typedef struct av1r_cycle {
    const av1r_frame_batch* const* const* batches;
    const int* count;
    int64_t* pos;
    int n_streams;
} av1r_cycle;
int av1r_cycle_next(void* user, int stream, const av1r_frame_batch** batch);
/* Source over IVF files (one per stream, caller-owned while the source lives): temporal
 * units parsed by the host parser (include/av1p.h) on the producer threads. */
int av1r_ivf_source_create(const uint8_t* const* files, const size_t* sizes, int n, av1r_stream_source* out);
void av1r_ivf_source_destroy(av1r_stream_source* src);

#ifdef __cplusplus
}
#endif
#endif
