"""ctypes mirror of include/av1r.h (the C-ABI batch structs).

Only the structs Python needs to build or inspect are mirrored; sizes are checked
against the C library's av1r_sizeof() at load time (see native.py) and in tests."""
import ctypes as C

AV1R_VERSION = 2

AV1R_OK = 0
AV1R_E_INVALID = -1
AV1R_E_UNSUPPORTED = -2
AV1R_E_DEVICE = -3
AV1R_E_NOMEM = -4
AV1R_E_NO_OUTPUT = -5

STAGE_RECON, STAGE_LF, STAGE_CDEF, STAGE_LR = 0, 1, 2, 3


class FrameHdr(C.Structure):
    _fields_ = [
        ("version", C.c_uint32),
        ("frame_width", C.c_int32), ("frame_height", C.c_int32),
        ("mi_cols", C.c_int32), ("mi_rows", C.c_int32),
        ("mi_stride", C.c_int32), ("mi_rows_alloc", C.c_int32),
        ("sb128", C.c_uint8), ("subx", C.c_uint8), ("suby", C.c_uint8), ("bitdepth", C.c_uint8),
        ("show_frame", C.c_uint8), ("show_existing_frame", C.c_uint8),
        ("frame_to_show", C.c_uint8), ("refresh_frame_flags", C.c_uint8),
        ("frame_type", C.c_uint8), ("enable_intra_edge_filter", C.c_uint8),
        ("force_integer_mv", C.c_uint8), ("allow_intrabc", C.c_uint8),
        ("ref_frame_idx", C.c_int8 * 8),
        ("gm_type", C.c_uint8 * 8),
        ("gm_params", (C.c_int32 * 6) * 8),
        ("ref_dist", C.c_uint8 * 8),
        ("delta_q_y_dc", C.c_int8), ("delta_q_u_dc", C.c_int8), ("delta_q_u_ac", C.c_int8),
        ("delta_q_v_dc", C.c_int8), ("delta_q_v_ac", C.c_int8),
        ("lf_level", C.c_uint8 * 4), ("lf_sharpness", C.c_uint8), ("lf_delta_enabled", C.c_uint8),
        ("delta_lf_multi", C.c_uint8),
        ("lf_ref_deltas", C.c_int8 * 8), ("lf_mode_deltas", C.c_int8 * 2),
        ("cdef_damping", C.c_uint8), ("cdef_bits", C.c_uint8),
        ("cdef_y_pri", C.c_uint8 * 8), ("cdef_y_sec", C.c_uint8 * 8),
        ("cdef_uv_pri", C.c_uint8 * 8), ("cdef_uv_sec", C.c_uint8 * 8),
        ("cdef_rows", C.c_int32), ("cdef_cols", C.c_int32),
        ("uses_lr", C.c_uint8), ("lr_type", C.c_uint8 * 3),
        ("lr_unit_size", C.c_int32 * 3),
        ("lr_unit_rows", C.c_int32 * 3), ("lr_unit_cols", C.c_int32 * 3),
        ("lr_unit_off", C.c_int32 * 3),
        ("reserved", C.c_uint8 * 16),
    ]


class FrameBatch(C.Structure):
    _fields_ = [
        ("hdr", C.c_void_p),
        ("mi", C.c_void_p),
        ("blocks", C.c_void_p), ("n_blocks", C.c_uint32),
        ("tbs", C.c_void_p), ("n_tbs", C.c_uint32),
        ("coefs", C.c_void_p), ("n_coefs", C.c_uint32),
        ("palette", C.c_void_p), ("n_palette", C.c_uint32),
        ("cdef_idx", C.c_void_p),
        ("lr_units", C.c_void_p), ("n_lr_units", C.c_uint32),
    ]


# record sizes (bytes) of the array element structs in av1r.h
SIZEOF_MI = 24
SIZEOF_BLOCK = 84
SIZEOF_TB = 20
SIZEOF_LR_UNIT = 12


# numpy record dtypes of the array structs (layouts of include/av1r.h)
import numpy as _np  # noqa: E402

MI_DTYPE = _np.dtype([
    ("mv", "<i2", (2, 2)), ("ref_frame", "i1", (2,)), ("mi_size", "u1"), ("y_mode", "u1"),
    ("filt", "u1"), ("flags", "u1"), ("lf_tx", "u1", (3,)), ("delta_lf", "i1", (4,)),
    ("uv_mode", "u1"), ("pad", "u1", (2,))])
BLOCK_DTYPE = _np.dtype([
    ("mi_row", "<u2"), ("mi_col", "<u2"), ("mi_size", "u1"), ("qindex", "u1"), ("y_mode", "u1"),
    ("uv_mode", "u1"), ("angle_delta_y", "i1"), ("angle_delta_uv", "i1"), ("filter_intra_mode", "u1"),
    ("cfl_alpha_u", "i1"), ("cfl_alpha_v", "i1"), ("palette_size_y", "u1"), ("palette_size_uv", "u1"),
    ("motion_mode", "u1"), ("compound_type", "u1"), ("interintra_mode", "u1"), ("wedge_index", "u1"),
    ("wedge_sign", "u1"), ("mask_type", "u1"), ("ii_edge", "u1"), ("pad0", "u1", (2,)), ("flags", "<u4"),
    ("max_luma_w", "<u2"), ("max_luma_h", "<u2"), ("local_warp", "<i4", (6,)), ("palette_off", "<u4"),
    ("first_tb", "<u4"), ("n_tbs", "<u4"), ("mv", "<i2", (2, 2)), ("ref_frame", "i1", (2,)), ("filt", "u1"),
    ("pad1", "u1"), ("delta_lf", "i1", (4,))])
TB_DTYPE = _np.dtype([
    ("block", "<u4"), ("coef_off", "<u4"), ("x", "<u2"), ("y", "<u2"), ("coef_cnt", "<u2"),
    ("plane", "u1"), ("tx_size", "u1"), ("tx_type", "u1"), ("flags", "u1"), ("pad", "u1", (2,))])
LR_DTYPE = _np.dtype([
    ("type", "u1"), ("sgr_set", "u1"), ("sgr_xqd", "i1", (2,)), ("wiener", "i1", (2, 3)), ("pad", "u1", (2,))])
assert MI_DTYPE.itemsize == SIZEOF_MI and BLOCK_DTYPE.itemsize == SIZEOF_BLOCK
assert TB_DTYPE.itemsize == SIZEOF_TB and LR_DTYPE.itemsize == SIZEOF_LR_UNIT
