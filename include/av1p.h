/*
 * av1p.h -- C-ABI of the host AV1 parser: OBUs in, av1r frame batches (av1r.h) out.
 *
 * The parse half of the reference decoder (oddstone/av1dec) as a library: what
 * Decoder::decode (decoder/Av1Decoder.cpp:49-109) does up to the point where it hands a
 * parsed frame to reconstruction (Decoder::decodeFrame, Av1Decoder.cpp:128-156).  Each
 * temporal unit yields zero or more frame batches in decode order -- decoded frames and
 * show_existing_frame records -- ready for av1r_decode_frame / av1r_pack /
 * av1r_show_existing.  Pure host code (no device, no HIP): contexts are independent, one
 * context must not be used from two threads at once.
 *
 * Entry points replace (reference file:line):
 *   av1p_create / av1p_destroy  -- Parser::Parser / ~Parser (decoder/Parser.h:642-680)
 *   av1p_decode_tu              -- the OBU loop of Decoder::decode (Av1Decoder.cpp:49-109)
 *                                  with Parser::parseSequenceHeader / parseFrameHeader /
 *                                  parseTileGroup and Tile::parse (Tile.cpp:122-160)
 *   av1p_frame                  -- the parsed frame the reference walks in decodeFrame
 *   av1p_set_tile_threads       -- (no counterpart: the reference parses tiles one after
 *                                  another, Parser::parseTileGroup, Parser.cpp:492-521)
 *   av1p_set_mode_info          -- (no counterpart: refdump.cpp fillFrameTables always
 *                                  builds the grid)
 *   av1p_set_frame_generations  -- (no counterpart: the reference decodes a frame before
 *                                  parsing the next)
 */
#ifndef AV1P_H
#define AV1P_H

#include <stddef.h>
#include <stdint.h>

#include "av1r.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct av1p_ctx av1p_ctx;

int av1p_create(av1p_ctx** out);
void av1p_destroy(av1p_ctx* ctx);
/* Parse one temporal unit (the payload of one IVF frame).  On success *n_frames receives
 * the number of frame batches it completed; they stay valid until the next call. */
int av1p_decode_tu(av1p_ctx* ctx, const uint8_t* data, size_t size, int* n_frames);
/* Frame batch i (0 <= i < n_frames) of the last av1p_decode_tu. */
const av1r_frame_batch* av1p_frame(av1p_ctx* ctx, int i);
/* Threads that parse the tiles of one frame concurrently (1: serial; default min(8, the
 * hardware threads), or the AV1P_TILE_THREADS environment variable).  Tiles are independent
 * for entropy decoding; the batch is identical whatever the setting. */
int av1p_set_tile_threads(av1p_ctx* ctx, int n);
/* 1 (default): each frame's av1r_frame_batch.mi holds the per-4x4 mode-info grid;
 * 0: mi is NULL. av1r_pack / av1r_decode_frame rebuild the grid on the device from the
 * block records and do not read it; av1r_frame_begin (tile-split decoding) needs it. */
int av1p_set_mode_info(av1p_ctx* ctx, int emit);
/* How long av1p_frame's batches stay valid: 1 (default) until the next av1p_decode_tu, 2
 * until the one after it (the frames of the previous unit are kept alive while the next
 * one is parsed: a consumer may still read them on another thread). */
int av1p_set_frame_generations(av1p_ctx* ctx, int n);
/* Message of the last failure (empty string if none). */
const char* av1p_last_error(av1p_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
