/* av1r_consts.h -- small AV1 enumerations and geometry tables (AV1 spec values; numeric
 * enum values as in the reference's aom/enums.h), shared by the HIP kernels, the CPU
 * oracle and the synthetic stream generator.  Larger normative tables: av1r_tables.h. */
#ifndef AV1R_CONSTS_H
#define AV1R_CONSTS_H
#include <stdint.h>
#include "av1r_tables.h"

/* BLOCK_SIZE */
enum {
    AV1R_BLOCK_4X4, AV1R_BLOCK_4X8, AV1R_BLOCK_8X4, AV1R_BLOCK_8X8, AV1R_BLOCK_8X16,
    AV1R_BLOCK_16X8, AV1R_BLOCK_16X16, AV1R_BLOCK_16X32, AV1R_BLOCK_32X16, AV1R_BLOCK_32X32,
    AV1R_BLOCK_32X64, AV1R_BLOCK_64X32, AV1R_BLOCK_64X64, AV1R_BLOCK_64X128, AV1R_BLOCK_128X64,
    AV1R_BLOCK_128X128, AV1R_BLOCK_4X16, AV1R_BLOCK_16X4, AV1R_BLOCK_8X32, AV1R_BLOCK_32X8,
    AV1R_BLOCK_16X64, AV1R_BLOCK_64X16, AV1R_BLOCK_SIZES
};
/* TX_SIZE */
enum {
    AV1R_TX_4X4, AV1R_TX_8X8, AV1R_TX_16X16, AV1R_TX_32X32, AV1R_TX_64X64, AV1R_TX_4X8,
    AV1R_TX_8X4, AV1R_TX_8X16, AV1R_TX_16X8, AV1R_TX_16X32, AV1R_TX_32X16, AV1R_TX_32X64,
    AV1R_TX_64X32, AV1R_TX_4X16, AV1R_TX_16X4, AV1R_TX_8X32, AV1R_TX_32X8, AV1R_TX_16X64,
    AV1R_TX_64X16, AV1R_TX_SIZES
};
/* TX_TYPE */
enum {
    AV1R_DCT_DCT, AV1R_ADST_DCT, AV1R_DCT_ADST, AV1R_ADST_ADST, AV1R_FLIPADST_DCT,
    AV1R_DCT_FLIPADST, AV1R_FLIPADST_FLIPADST, AV1R_ADST_FLIPADST, AV1R_FLIPADST_ADST,
    AV1R_IDTX, AV1R_V_DCT, AV1R_H_DCT, AV1R_V_ADST, AV1R_H_ADST, AV1R_V_FLIPADST,
    AV1R_H_FLIPADST
};
/* PREDICTION_MODE */
enum {
    AV1R_DC_PRED, AV1R_V_PRED, AV1R_H_PRED, AV1R_D45_PRED, AV1R_D135_PRED, AV1R_D113_PRED,
    AV1R_D157_PRED, AV1R_D203_PRED, AV1R_D67_PRED, AV1R_SMOOTH_PRED, AV1R_SMOOTH_V_PRED,
    AV1R_SMOOTH_H_PRED, AV1R_PAETH_PRED, AV1R_NEARESTMV, AV1R_NEARMV, AV1R_GLOBALMV,
    AV1R_NEWMV, AV1R_NEAREST_NEARESTMV, AV1R_NEAR_NEARMV, AV1R_NEAREST_NEWMV,
    AV1R_NEW_NEARESTMV, AV1R_NEAR_NEWMV, AV1R_NEW_NEARMV, AV1R_GLOBAL_GLOBALMV, AV1R_NEW_NEWMV
};
#define AV1R_UV_CFL_PRED 13
enum { AV1R_SIMPLE_TRANSLATION, AV1R_OBMC_CAUSAL, AV1R_LOCALWARP };
enum { AV1R_II_DC_PRED, AV1R_II_V_PRED, AV1R_II_H_PRED, AV1R_II_SMOOTH_PRED };
enum {
    AV1R_COMPOUND_WEDGE, AV1R_COMPOUND_DIFFWTD, AV1R_COMPOUND_AVERAGE, AV1R_COMPOUND_INTRA,
    AV1R_COMPOUND_DISTANCE
};
enum { AV1R_EIGHTTAP, AV1R_EIGHTTAP_SMOOTH, AV1R_EIGHTTAP_SHARP, AV1R_BILINEAR };
enum { AV1R_GM_IDENTITY, AV1R_GM_TRANSLATION, AV1R_GM_ROTZOOM, AV1R_GM_AFFINE };
enum { AV1R_RESTORE_NONE, AV1R_RESTORE_WIENER, AV1R_RESTORE_SGRPROJ, AV1R_RESTORE_SWITCHABLE };
#define AV1R_NONE_FRAME (-1)
#define AV1R_INTRA_FRAME 0
#define AV1R_MAX_FRAME_DISTANCE 31

#if defined(__HIP_DEVICE_COMPILE__)
#define AV1R_CT __device__ __constant__
#else
#define AV1R_CT
#endif

static const AV1R_CT uint8_t av1r_num4x4w[AV1R_BLOCK_SIZES] = {1, 1, 2, 2, 2, 4, 4, 4, 8, 8, 8, 16, 16, 16, 32, 32, 1, 4, 2, 8, 4, 16};
static const AV1R_CT uint8_t av1r_num4x4h[AV1R_BLOCK_SIZES] = {1, 2, 1, 2, 4, 2, 4, 8, 4, 8, 16, 8, 16, 32, 16, 32, 4, 1, 8, 2, 16, 4};
static const AV1R_CT uint8_t av1r_miw_log2[AV1R_BLOCK_SIZES] = {0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 4, 4, 4, 5, 5, 0, 2, 1, 3, 2, 4};
static const AV1R_CT uint8_t av1r_mih_log2[AV1R_BLOCK_SIZES] = {0, 1, 0, 1, 2, 1, 2, 3, 2, 3, 4, 3, 4, 5, 4, 5, 2, 0, 3, 1, 4, 2};
/* Subsampled_Size[bsize][1][1] (4:2:0), Parser.cpp:412-435 */
static const AV1R_CT uint8_t av1r_ss420[AV1R_BLOCK_SIZES] = {0, 0, 0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 1, 2, 16, 17, 18, 19};
/* Wedge_Bits[bsize] (InterPredict.cpp:752-755) */
static const AV1R_CT uint8_t av1r_wedge_bits[AV1R_BLOCK_SIZES] = {0, 0, 0, 4, 4, 4, 4, 4, 4, 4, 0, 0, 0, 0, 0, 0, 0, 0, 4, 4, 0, 0};

static const AV1R_CT uint8_t av1r_tx_w[AV1R_TX_SIZES] = {4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64};
static const AV1R_CT uint8_t av1r_tx_h[AV1R_TX_SIZES] = {4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16};
static const AV1R_CT uint8_t av1r_tx_w_log2[AV1R_TX_SIZES] = {2, 3, 4, 5, 6, 2, 3, 3, 4, 4, 5, 5, 6, 2, 4, 3, 5, 4, 6};
static const AV1R_CT uint8_t av1r_tx_h_log2[AV1R_TX_SIZES] = {2, 3, 4, 5, 6, 3, 2, 4, 3, 5, 4, 6, 5, 4, 2, 5, 3, 6, 4};
/* Transform_Row_Shift (TransformBlock.cpp:2168-2171) */
static const AV1R_CT uint8_t av1r_tx_row_shift[AV1R_TX_SIZES] = {0, 1, 2, 2, 2, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2};

/* Mode_To_Angle (IntraPredict.cpp:173) */
static const AV1R_CT uint8_t av1r_mode_to_angle[13] = {0, 90, 180, 45, 135, 113, 157, 203, 67, 0, 0, 0, 0};
/* Intra_Edge_Kernel (IntraPredict.cpp:318-322) */
static const AV1R_CT uint8_t av1r_edge_kernel[3][5] = {{0, 4, 8, 4, 0}, {0, 5, 6, 5, 0}, {2, 4, 4, 4, 2}};
/* Filter_Intra_Mode_To_Intra_Dir is not needed: filter intra is a separate predictor. */

/* get_obmc_mask (InterPredict.cpp:630-656), concatenated: len 2 @0, 4 @2, 8 @6, 16 @14, 32 @30 */
static const AV1R_CT uint8_t av1r_obmc_mask[62] = {
    45, 64,
    39, 50, 59, 64,
    36, 42, 48, 53, 57, 61, 64, 64,
    34, 37, 40, 43, 46, 49, 52, 54, 56, 58, 60, 61, 64, 64, 64, 64,
    33, 35, 36, 38, 40, 41, 43, 44, 45, 47, 48, 50, 51, 52, 53, 55,
    56, 57, 58, 59, 60, 60, 61, 62, 64, 64, 64, 64, 64, 64, 64, 64};
/* Quant_Dist_Weight / Quant_Dist_Lookup (InterPredict.cpp:919-930) */
static const AV1R_CT uint8_t av1r_quant_dist_weight[4][2] = {{2, 3}, {2, 5}, {2, 7}, {1, AV1R_MAX_FRAME_DISTANCE}};
static const AV1R_CT uint8_t av1r_quant_dist_lookup[4][2] = {{9, 7}, {11, 5}, {12, 4}, {13, 3}};

/* Wedge directions and codebook (InterPredict.cpp:730-830) */
enum { AV1R_WEDGE_HORIZONTAL, AV1R_WEDGE_VERTICAL, AV1R_WEDGE_OBLIQUE27, AV1R_WEDGE_OBLIQUE63,
       AV1R_WEDGE_OBLIQUE117, AV1R_WEDGE_OBLIQUE153 };
static const AV1R_CT uint8_t av1r_wedge_codebook[3][16][3] = {
    {{2, 4, 4}, {3, 4, 4}, {4, 4, 4}, {5, 4, 4}, {0, 4, 2}, {0, 4, 4}, {0, 4, 6}, {1, 4, 4},
     {2, 4, 2}, {2, 4, 6}, {5, 4, 2}, {5, 4, 6}, {3, 2, 4}, {3, 6, 4}, {4, 2, 4}, {4, 6, 4}},
    {{2, 4, 4}, {3, 4, 4}, {4, 4, 4}, {5, 4, 4}, {1, 2, 4}, {1, 4, 4}, {1, 6, 4}, {0, 4, 4},
     {2, 4, 2}, {2, 4, 6}, {5, 4, 2}, {5, 4, 6}, {3, 2, 4}, {3, 6, 4}, {4, 2, 4}, {4, 6, 4}},
    {{2, 4, 4}, {3, 4, 4}, {4, 4, 4}, {5, 4, 4}, {0, 4, 2}, {0, 4, 6}, {1, 2, 4}, {1, 6, 4},
     {2, 4, 2}, {2, 4, 6}, {5, 4, 2}, {5, 4, 6}, {3, 2, 4}, {3, 6, 4}, {4, 2, 4}, {4, 6, 4}}};

/* CDEF (Cdef.cpp:60-65, 120-140, 200-202) */
static const AV1R_CT uint8_t av1r_cdef_uv_dir420[8] = {0, 1, 2, 3, 4, 5, 6, 7}; /* Cdef_Uv_Dir[1][1] (identity) */
static const AV1R_CT int8_t av1r_cdef_directions[8][2][2] = {
    {{-1, 1}, {-2, 2}}, {{0, 1}, {-1, 2}}, {{0, 1}, {0, 2}}, {{0, 1}, {1, 2}},
    {{1, 1}, {2, 2}}, {{1, 0}, {2, 1}}, {{1, 0}, {2, 0}}, {{1, 0}, {2, -1}}};
static const AV1R_CT uint8_t av1r_cdef_pri_taps[2][2] = {{4, 2}, {3, 3}};
static const AV1R_CT uint8_t av1r_cdef_sec_taps[2][2] = {{2, 1}, {2, 1}};
static const AV1R_CT int16_t av1r_cdef_div_table[9] = {0, 840, 420, 280, 210, 168, 140, 120, 105};

/* Sgr_Params (Av1Common.h:206-211) */
static const AV1R_CT uint8_t av1r_sgr_params[16][4] = {
    {2, 12, 1, 4}, {2, 15, 1, 6}, {2, 18, 1, 8}, {2, 21, 1, 9}, {2, 24, 1, 10}, {2, 29, 1, 11},
    {2, 36, 1, 12}, {2, 45, 1, 13}, {2, 56, 1, 14}, {2, 68, 1, 15}, {0, 0, 1, 5}, {0, 0, 1, 8},
    {0, 0, 1, 11}, {0, 0, 1, 14}, {2, 30, 0, 0}, {2, 75, 0, 0}};

#endif
