/*
 * av1dec.h -- C-ABI of the whole decoder: bitstream in, I420 frames out.
 *
 * The reference's top-level API (YamiAv1::Decoder, decoder/Av1Decoder.h:47-70) for FFI
 * callers: the C++ class in include/YamiAv1/Av1Decoder.h is a thin wrapper over these.
 *   av1d_create / av1d_destroy -- Decoder::Decoder / ~Decoder (Av1Decoder.cpp:40-47)
 *   av1d_decode                -- Decoder::decode (Av1Decoder.cpp:49-109): parse one temporal
 *                                 unit (include/av1p.h), reconstruct + filter each frame on
 *                                 the GPU (include/av1r.h), queue shown frames
 *   av1d_output_size / av1d_get_output
 *                              -- Decoder::getOutput (Av1Decoder.cpp:203-211) + the I420 copy
 *                                 of DecodeOutput::output (tests/DecodeOutput.cpp:48-69)
 */
#ifndef AV1DEC_H
#define AV1DEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct av1d_ctx av1d_ctx;

int av1d_create(int device, av1d_ctx** out);
void av1d_destroy(av1d_ctx* ctx);
/* Status codes are those of av1r.h (AV1R_OK, AV1R_E_*). */
int av1d_decode(av1d_ctx* ctx, const uint8_t* data, size_t size);
/* Dimensions of the next frame getOutput would return: AV1R_E_NO_OUTPUT if none. */
int av1d_output_size(av1d_ctx* ctx, int* width, int* height);
/* Copy the next shown frame's visible I420 planes and pop it (AV1R_E_NO_OUTPUT if none). */
int av1d_get_output(av1d_ctx* ctx, uint8_t* y, int y_stride, uint8_t* u, int u_stride, uint8_t* v,
                    int v_stride, int* width, int* height);
/* Drop every decoded frame not yet returned (IVideoDecoder::flush, a seek): the next unit
 * should start at a key frame. */
int av1d_flush(av1d_ctx* ctx);
const char* av1d_last_error(av1d_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
