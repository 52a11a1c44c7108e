// av1r_dev.h -- shared device-side definitions of the gfx950 reconstruction backend.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "av1r.h"
#include "av1r_consts.h"

#define DEV __device__ __forceinline__

// XCD-aware workgroup order (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement"):
// workgroups are dealt round-robin over the 8 XCDs, so b and b + 8 share one XCD's L2.
// Renumbering gives each XCD a contiguous eighth of the grid's logical order instead of
// every eighth tile: neighbouring tiles (reference windows around the same motion, filter
// halos) and, in a batched launch, one frame's tiles stay in one L2.  Speed only: it is a
// bijection on [0, g), so any placement stays correct.
#ifndef AV1R_XCD_ORDER
#define AV1R_XCD_ORDER 1
#endif
DEV uint32_t xcd_order(uint32_t b, uint32_t g)
{
#if AV1R_XCD_ORDER
    const uint32_t x = b & 7, q = g >> 3, r = g & 7;
    return x * q + (x < r ? x : r) + (b >> 3);
#else
    (void)g;
    return b;
#endif
}
// This workgroup's logical (x, y, z) in XCD order (x fastest, as the hardware deals them).
DEV uint3 xcd_block()
{
    const uint32_t gxy = gridDim.x * gridDim.y;
    uint32_t L = xcd_order(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), gxy * gridDim.z);
    uint3 r;
    r.z = L / gxy;
    L -= r.z * gxy;
    r.y = L / gridDim.x;
    r.x = L - r.y * gridDim.x;
    return r;
}

// The same within each z slice only (z = blockIdx.z): every XCD takes a contiguous eighth of
// every slice.  For grids whose slices carry unequal work (k_lr: z = frame x plane, chroma
// slices half empty) a contiguous eighth of the whole grid would leave the XCDs holding
// luma slices with most of the work.
DEV uint3 xcd_block_xy()
{
    const uint32_t gxy = gridDim.x * gridDim.y;
    const uint32_t L = xcd_order(blockIdx.x + gridDim.x * blockIdx.y, gxy);
    uint3 r;
    r.z = blockIdx.z;
    r.y = L / gridDim.x;
    r.x = L - r.y * gridDim.x;
    return r;
}

// One plane of a device frame.  Frames are SB-aligned + 64 px margin, origin at (0,0);
// w/h are the VISIBLE plane dims (YuvFrame::widths/heights, VideoFrame.cpp:49-51).
struct DevPlane {
    uint8_t* p;
    int stride;
    int w, h;
};
struct DevFrame {
    DevPlane pl[3];
    int width, height;  // FrameWidth / FrameHeight of the frame stored here
};

// One work item of a frame's level-ordered schedule (built by the host, 32 bytes: one
// scalar load gives a transform block everything it needs before its block record).
struct WorkItem {
    uint32_t code;      // AV1R_ITEM(kind, index)
    uint32_t block;     // owning block
    uint32_t coef_off;  // TB: first coefficient
    uint16_t x, y;      // TB: plane position
    uint16_t coef_cnt;  // TB
    uint8_t plane, tx_size, tx_type, flags;  // TB (flags: AV1R_TB_*)
    uint8_t pred;       // TB prediction source: AV1R_PRED_INTRA / _PALETTE / _INTER
    uint8_t pub;        // k_flow: 1 = a dependency list names this item (store sc1, drain, flag)
    uint16_t dep_cnt;   // k_flow: the items whose pixels this one reads ...
    uint16_t hflags;    // host only (build_schedule -> pack_frame): AV1R_WI_TINY
    uint32_t dep_off;   // ... at KParams::deps[dep_off, dep_off + dep_cnt) (item positions)
};
static_assert(sizeof(WorkItem) == 32, "WorkItem layout");
#define AV1R_PRED_INTRA 0
#define AV1R_PRED_PALETTE 1
#define AV1R_PRED_INTER 2
#define AV1R_WI_TINY 1u

// k_flow's tiny items (round 6).  An intra transform block of at most 8x8 on the lean path
// (intra_fast.h: not palette, not filter-intra) in a frame with edge granules, on a crowded
// level, is described whole in the 32 bytes of its WorkItem slot: every parameter fi_setup
// derives (the prediction class, edge-filter strengths and lengths, upsampling, dx / dy,
// CFL's alpha and luma extent), its granule masks and residual tile.  k_flow runs them four
// to a wave, 16 lanes each (tiny_run, recon.hip): one scalar load per item gives all it
// needs, and the four items' memory round trips overlap.  build_schedule marks the items
// AV1R_WI_TINY (the tiny groups of a level, up to 16 items, group flag FLOW_G_TINY, come
// before its other small items) and k_mi_zero rewrites their slots on the device
// (tiny_from_item, filters.hip: no host time).  Bytes 26-27 -- WorkItem::hflags -- stay 0, so
// a rewritten slot is not rewritten again when a prepared frame is decoded twice.
struct TinyItem {
    uint16_t x, y;      // plane position
    uint8_t shape;      // plane (bits 0-1) | log2W - 2 (bit 2) | log2H - 2 (bit 3) | class (bits 4-7, FI_*)
    uint8_t flags;      // TI_*
    uint8_t str;        // edge-filter strengths: above | left << 4
    uint8_t lim;        // aboveLimit - x | (leftLimit - y) << 4
    uint8_t nA, nL;     // edge-filter lengths (numPx + 1)
    uint8_t nUA, nUL;   // upsampled lengths (0: none)
    uint8_t masks;      // granule masks: above run (bits 0-3) | left run << 4
    uint8_t mC;         // corner: bit 0 written in the launch, bit 1 its owner's right column
    uint16_t p0, p1;    // directional: dx, dy; CFL: max_luma_w, max_luma_h
    int8_t alpha;       // CFL
    uint8_t pad;
    uint32_t dep_off;   // dependency list (CFL's co-located luma) at KParams::deps[dep_off ..)
    uint16_t dep_cnt;
    uint16_t zero;      // (WorkItem::hflags' bytes: 0)
    uint32_t res;       // residual tile (int16 elements into KParams::res; ~0u: none)
};
static_assert(sizeof(TinyItem) == 32, "TinyItem layout");
static_assert(offsetof(TinyItem, zero) == offsetof(WorkItem, hflags), "TinyItem / WorkItem overlay");
#define TI_HA 1u
#define TI_HL 2u
#define TI_CFL 4u
#define TI_CORNER 8u
#define TI_PUB 16u
#define FLOW_G_TINY 0x40u  // k_flow group descriptor: n | FLOW_G_TINY = n tiny items
#define FLOW_TINY_G 16     // tiny items per group (four per wave)
// the lean path's prediction classes (intra_fast.h fi_setup; TinyItem::shape)
enum { FI_DC = 0, FI_V, FI_H, FI_Z1, FI_Z2, FI_Z3, FI_SMOOTH, FI_SMOOTH_V, FI_SMOOTH_H, FI_PAETH };

// The device's block record: the fields of av1r_block that the kernels read, packed (52 bytes
// against 84: a 1080p inter frame uploads ~0.45 MB less).  Left out, into KParams::bext at
// index palette_off (a palette block is never inter, so the field is free for the inter
// blocks that need it): the 24-byte local-warp parameters of an AV1R_BLK_LOCAL_VALID block
// and the transform-block range of an AV1R_BLK_INTERINTRA block (k_flow's ii_item adds
// its residuals), 8 words each: LocalWarpParams[6], first_tb, n_tbs.  Every other kernel
// reaches a TB's block, never the reverse.  Written by pack_frame (av1r_host.cpp).
struct DevBlock {
    // av1r_block's first 32 bytes, as they are
    uint16_t mi_row, mi_col;
    uint8_t mi_size, qindex, y_mode, uv_mode;
    int8_t angle_delta_y, angle_delta_uv;
    uint8_t filter_intra_mode;
    int8_t cfl_alpha_u, cfl_alpha_v;
    uint8_t palette_size_y, palette_size_uv;
    uint8_t motion_mode, compound_type, interintra_mode, wedge_index, wedge_sign, mask_type, ii_edge;
    uint8_t pad0[2];
    uint32_t flags;
    uint16_t max_luma_w, max_luma_h;
    uint32_t palette_off;  // palette blocks: their palette record; LOCAL_VALID / INTERINTRA blocks: their bext index
    // av1r_block's last 16 bytes, as they are
    int16_t mv[2][2];
    int8_t ref_frame[2];
    uint8_t filt;
    uint8_t pad1;
    int8_t delta_lf[4];
};
static_assert(sizeof(DevBlock) == 52, "DevBlock layout");
static_assert(offsetof(av1r_block, max_luma_h) == 30 && offsetof(DevBlock, max_luma_h) == 30, "DevBlock head");
static_assert(offsetof(av1r_block, mv) + 16 == sizeof(av1r_block) && offsetof(DevBlock, mv) + 16 == sizeof(DevBlock),
    "DevBlock tail");

// The device's transform-block record (16 bytes against av1r_tb's 20, pack_frame): the
// same fields, the small ones as bit-fields, and the coefficient width: a TB whose levels all
// fit 6 signed bits (nearly every one) keeps its coefficients as 16-bit words in
// KParams::coefs16, the others as av1r_tb's 32-bit words in KParams::coefs (coef_off indexes
// the array its width selects; coef_at below reads either as the 32-bit form).
#define AV1R_TBD_WIDE 16u  // flags bit (device only; WorkItem::flags too)
struct DevTb {
    uint32_t block;
    uint32_t coef_off;
    uint16_t x, y;
    uint16_t coef_cnt;
    uint16_t plane : 2, tx_size : 5, tx_type : 4, flags : 5;
};
static_assert(sizeof(DevTb) == 16, "DevTb layout");

// Everything the stage kernels read about one frame.  A launch covers n frames (one per
// stream of a batch): the kernels receive a device array of n KParams and pick theirs
// by blockIdx (see k_level / k_lf / k_cdef / k_lr).
struct KParams {
    const av1r_frame_hdr* hdr;
    const av1r_mi* mi;
    const DevBlock* blocks;
    const int32_t* bext;  // LOCAL_VALID / INTERINTRA blocks' warp parameters and TB range, 8 words each (DevBlock)
    const DevTb* tbs;
    const uint32_t* coefs;    // the coefficients of the wide TBs (AV1R_TBD_WIDE), av1r_tb's form
    const uint16_t* coefs16;  // everyone else's: (level << 10 | pos) as int16 (|level| < 32)
    const uint8_t* palette;
    const int8_t* cdef_idx;
    const av1r_lr_unit* lr;
    const WorkItem* items;  // this frame's level-ordered work items (transform blocks, inter-intra blends)
    const uint32_t* tiles;  // its inter tiles, level-ordered: AV1R_ITEM(AV1R_ITEM_INTER, block << 4 | row << 2 | col)
    const uint32_t* deps;   // k_flow: dependency lists (positions in items)
    uint32_t* done;         // k_flow: per item, the epoch of the launch that completed it
    // k_flow mode: residuals precomputed by k_resid.  tb_res[tb]: the TB's residual tile
    // (w x h int16, row-major) at res + tb_res[tb], or ~0u (no coefficients, or an inter
    // TB outside an inter-intra block: k_resid adds it into the frame directly)
    const uint32_t* tb_res;
    int16_t* res;
    const uint32_t* resid_s;  // TBs with coefficients and sides <= 16: n_resid_t workgroups of 64 4x4 TBs, n_resid_e of 32 TBs <= 8x8, then 16 per workgroup (~0u pads)
    const uint32_t* resid_l;  // the larger ones: [nm][nm workgroups of two TBs <= 32x32 (~0u pads)][then one per workgroup]
    // k_flow edge granules (cdna_hip_programming.md §6 Guideline 16 R2: the data is the
    // flag).  Per plane and 4x4 unit, the unit's bottom row (gran_h[row * gw + col]) and
    // right column (gran_v[col * gh + row], top to bottom) as {4 pixels, epoch << 32},
    // stored by the k_flow item that writes the unit.  gran = 0: edges through dependency
    // flags instead (every edge owner in the item's list)
    uint64_t* gran_h[3];
    uint64_t* gran_v[3];
    int gran_w[3], gran_hn[3];
    int gran;
    int fi;  // k_flow: small intra TBs take the lean path (intra_fast.h; AV1R_FI=0: off)
    uint32_t n_items;
    uint32_t n_resid_t;     // k_resid_s: workgroups of 4x4 TBs heading resid_s
    uint32_t n_resid_e;     // k_resid_s: then workgroups of 32 TBs with both sides <= 8
    uint32_t trace_base;    // -DAV1R_TRACE, k_flow mode: this frame's first timeline row
    int mi_stride;
    int mi_cols, mi_rows;
    int mi_rows_alloc;
    uint32_t n_blocks, n_tbs;  // k_mi: the records the mode-info grid is derived from
    int frame_w, frame_h;
    DevFrame cur;     // frame under reconstruction (k_lf: deblocked in place)
    DevFrame dbk;     // the deblocked frame (k_lf deblocks cur in place: cur)
    DevFrame cdef;    // CDEF output (Cdef::filter's copy, Cdef.cpp:43)
    DevFrame lrout;   // loop-restoration output (LoopRestoration.cpp:216)
    DevFrame ref[8];  // reference store slots
};
// (resid_l carries its own class count at its head rather than a KParams field: a field
// changed every kernel's code through the field offsets and the per-frame KParams stride,
// which made the filters' A/B readings hard to attribute -- round 6, profiles/r06_ab_residm.txt)
static_assert(sizeof(KParams) == 1232, "KParams layout");

// Coefficient q of a TB whose first coefficient is `off` (DevTb / WorkItem coef_off), in
// av1r_tb's 32-bit form: a 16-bit word (level << 10 | pos, |level| < 32) sign-extends to it.
DEV uint32_t coef_at(const KParams& k, uint32_t off, uint32_t flags, int q)
{
    return (flags & AV1R_TBD_WIDE) ? k.coefs[off + q] : (uint32_t)(int32_t)(int16_t)k.coefs16[off + q];
}

// launch batches: at most AV1R_MAX_BATCH frames per launch
#define AV1R_MAX_BATCH 32

// The frames' parameters of a launch live at the start of its metadata buffer (uploaded
// with one copy per batch) and are read through the constant address space: every field
// is a scalar load the compiler may hoist anywhere (behind a plain global pointer the same
// struct costs ~100 VGPRs of hoisted vector loads in k_inter, and the filters reload it
// inside their pixel loops because the pixel stores might alias it).
typedef const __attribute__((address_space(4))) KParams* KpConst;
#define KP(kps, i) (*(const KParams*)(&((KpConst)(kps))[i]))

// k_flow control block (recon.hip): FLOW_QUEUES queue heads, one 128-B line each, then
// the error word, the address of the host's error word and the spin bound (one line),
// then the queue-assignment counter (its own line); written by the host before every launch
#define FLOW_QUEUES 8
#define FLOW_LINE 32
#define FLOW_ERR (FLOW_QUEUES * FLOW_LINE)
#define FLOW_HOSTERR (FLOW_ERR + 2)  // (8 bytes) address of the launch's pinned host error word
#define FLOW_SPINLIM (FLOW_ERR + 4)  // polls before a wait gives up (0: FLOW_SPINS)
#define FLOW_ASSIGN (FLOW_ERR + FLOW_LINE)  // workgroup entries: entry k serves queue k % FLOW_QUEUES
#define FLOW_CTL_BYTES (4 * (FLOW_ASSIGN + FLOW_LINE))
// k_flow spin bound, in polls of running waves (each a global load round trip, ~0.5-2 us),
// not in wall-clock time: a wave that the hardware preempts (context save / restore) does
// not count the time it was off the chip, so only a wait that makes no progress WHILE
// running gives up (~2-6 s), or one outliving FLOW_WALL
#define FLOW_SPINS (1u << 22)
#define FLOW_WALL 3000000000ull  // 30 s of the 100 MHz real-time counter
// the launch's spin bound (av1r_set_flow_spins: a test forces the timeout path with 1)
#ifndef AV1R_ERR_POLL_MASK
#define AV1R_ERR_POLL_MASK 31  // spinning waves read the launch's error word every 32nd poll
#endif
DEV uint32_t flow_spin_limit(const uint32_t* ctl)
{
    const uint32_t v = __hip_atomic_load(ctl + FLOW_SPINLIM, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v ? v : FLOW_SPINS;
}

#define CLIP3(lo, hi, v) ((v) < (lo) ? (lo) : ((v) > (hi) ? (hi) : (v)))
DEV int clip1(int v) { return CLIP3(0, 255, v); }
// log2 of a power of two (block, tile, prediction-unit and transform sides): the per-lane
// loops over a w-wide region index rows by shifts, not by an integer division (~12 VALU ops)
DEV int ilog2p(int x) { return 31 - __builtin_clz((unsigned)x); }
DEV int r2(int x, int n) { return n == 0 ? x : ((x + (1 << (n - 1))) >> n); }
DEV int r2s(int x, int n) { return x >= 0 ? r2(x, n) : -r2(-x, n); }
DEV int64_t r2_64(int64_t x, int n) { return n == 0 ? x : ((x + ((int64_t)1 << (n - 1))) >> n); }
DEV int64_t r2s_64(int64_t x, int n) { return x >= 0 ? r2_64(x, n) : -r2_64(-x, n); }
DEV int iabs(int v) { return v < 0 ? -v : v; }
DEV int imin(int a, int b) { return a < b ? a : b; }
DEV int imax(int a, int b) { return a > b ? a : b; }
DEV int floor_log2_u64(uint64_t x) { return x ? 63 - __builtin_clzll(x) : -1; }
DEV int floor_log2(int x) { return x > 0 ? 31 - __builtin_clz((unsigned)x) : -1; }

// Cooperating lanes of one work item: the whole workgroup (NT = blockDim.x = 256), one
// wave (NT = 64, several items per workgroup), or a 16-lane quarter of a wave (NT = 16,
// k_resid_s).  Below a workgroup, synchronisation is wave-level: a wave's LDS operations
// complete in order, so only the compiler must not reorder.
template <int NT>
DEV int coop_lane()
{
    // opaque to the optimiser: in k_flow's persistent loop, lane-derived addresses would
    // otherwise be hoisted out of the loop for every code path and kept live (2x VGPRs)
    int t = NT >= 256 ? (int)threadIdx.x : (int)(threadIdx.x & (NT - 1));
    asm volatile("" : "+v"(t));
    return t;
}
template <int NT>
DEV void coop_sync()
{
    if (NT <= 64) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

// Wave-uniform reads of data no kernel of the launch writes (the batch's records, the
// spec tables) through the scalar cache.  A global_load of a uniform value is a VECTOR
// memory op: its s_waitcnt vmcnt counts every store the wave issued before it (gfx9 keeps
// loads and stores in one in-order counter), so in k_flow each record or table
// read after an item's pixel stores waited for those stores to reach L2.  s_load (address
// space 4, lgkmcnt) does not.  Only for data final before the launch: the scalar cache is
// not coherent with vector stores (a dispatch's acquire invalidates it).
typedef __attribute__((address_space(4))) const uint32_t sc_u32;
DEV uintptr_t uniform_addr(const void* p)
{
    const uintptr_t a = (uintptr_t)p;
    // (readfirstlane returns int: through uint32_t, or a low word >= 2^31 sign-extends)
    return (uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a) |
           ((uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32);
}
template <class T>
DEV T sload(const T* p)  // a record (size and address multiples of 4)
{
    static_assert(sizeof(T) % 4 == 0, "sload: dword records");
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(4))) T*)uniform_addr(p);
#else
    return *p;  // (the host pass of the single-source compile; never run)
#endif
}
template <class T>
DEV int sfield(const T* p)  // a byte / halfword at a uniform address (the dword holding it)
{
    static_assert(sizeof(T) <= 2, "sfield: byte / halfword fields");
    const uintptr_t a = uniform_addr(p);
    const uint32_t w = *(sc_u32*)(a & ~(uintptr_t)3) >> (8 * (a & 3));
    return (int)(T)w;
}
// tab[i], the index clamped to the table: a scalar load also runs in a branch no lane
// takes (exec = 0), with whatever the index register holds there
template <class T, int N>
DEV int stab(const T (&tab)[N], int i)
{
    return sfield(tab + (i < 0 ? 0 : i >= N ? N - 1 : i));
}
template <int NT, class T, int N>
DEV int ctab(const T (&tab)[N], int i)  // tab[i] for an item of NT lanes: scalar when i is wave-uniform
{
    if constexpr (NT >= 64) return stab(tab, i);
    else return tab[i];
}

DEV const av1r_mi& mi_at(const KParams& k, int row, int col) { return k.mi[(size_t)row * k.mi_stride + col]; }
DEV int plane_bsize(int bs, int plane) { return plane ? av1r_ss420[bs] : bs; }
DEV uint8_t& px(const DevPlane& p, int x, int y) { return p.p[(size_t)y * p.stride + x]; }

// Pixel access of the frame under reconstruction.  COH = false: plain loads / stores (the
// level launches: every pixel an item reads was finalised by an earlier launch).  COH =
// true: agent-scope coherent accesses (global_load / global_store ... sc1) for the
// dataflow kernel k_flow, where producer and consumer items run in the SAME launch on
// different CUs / XCDs: sc1 stores write through to the device coherence point and sc1
// loads bypass the (never refreshed) vector L1, so after a producer's
// `s_waitcnt vmcnt(0)` + sc1 flag store (flow_publish) a consumer that has seen the flag
// (flow_wait) reads the final bytes.  x of the 4-byte forms is a multiple of 4.
template <bool COH>
DEV uint8_t ldp(const DevPlane& p, int x, int y)
{
    uint8_t* a = p.p + (size_t)y * p.stride + x;
    if constexpr (COH) return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *a;
}
template <bool COH>
DEV void stp(const DevPlane& p, int x, int y, uint8_t v)
{
    uint8_t* a = p.p + (size_t)y * p.stride + x;
    if constexpr (COH) __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *a = v;
}
template <bool COH>
DEV uint32_t ldp4(const DevPlane& p, int x, int y)
{
    uint32_t* a = reinterpret_cast<uint32_t*>(p.p + (size_t)y * p.stride + x);
    if constexpr (COH) return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *a;
}
template <bool COH>
DEV void stp4(const DevPlane& p, int x, int y, uint32_t v)
{
    uint32_t* a = reinterpret_cast<uint32_t*>(p.p + (size_t)y * p.stride + x);
    if constexpr (COH) __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *a = v;
}

// runtime choice between the two forms (a uniform branch): coh = sc1, else plain
DEV uint8_t ldp_c(const DevPlane& p, int x, int y, bool coh) { return coh ? ldp<true>(p, x, y) : ldp<false>(p, x, y); }
DEV uint32_t ldp4_c(const DevPlane& p, int x, int y, bool coh) { return coh ? ldp4<true>(p, x, y) : ldp4<false>(p, x, y); }
DEV void stp4_c(const DevPlane& p, int x, int y, uint32_t v, bool coh)
{
    if (coh) stp4<true>(p, x, y, v);
    else stp4<false>(p, x, y, v);
}
DEV void stp_c(const DevPlane& p, int x, int y, uint8_t v, bool coh)
{
    if (coh) stp<true>(p, x, y, v);
    else stp<false>(p, x, y, v);
}
// THE INVARIANT of the dataflow kernels.  k_flow: every read of a pixel that another item
// of the same launch may have written goes through the sc1 accessors (ldp<true> /
// ldp4<true>) or a granule, and every such pixel is stored sc1 -- a plain load could return
// a stale line from this CU's L1 (cdna_hip_programming.md §6 Guideline 16).  Checklist for a
// new read site in recon.hip's AV1R_FLOW_PART code (k_flow): (1) can another item of this
// launch have written the pixel?  If not (batch data, reference frames, pixels final before
// the launch), any load will do.  (2) If so: it is read through ldp<true>/ldp4<true> (or
// ldp_c/ldp4_c with coh = true) or arrives in a granule, after the wait that orders it.
// (3) Its writer stores it sc1 (stp4<true>,
// stp_c with coh), and publishes a granule or a done flag if a consumer's wait names it.
// The read sites today: gran_gather (intra_dev.h), tb_predict's CFL luma, fi_run's CFL
// luma (intra_fast.h) and ii_item's edges and inter prediction (recon.hip); each is marked
// "(flow read site)".  Scalar loads (sload / stab / sfield) are for batch data only.
// One deliberate exception: an intra edge is gathered whole, but the host names (masks /
// dependency lists) only the units the prediction mode uses (av1r_host.cpp intra_needs:
// above-right for zone 1, below-left for zone 3, the corner for Paeth / directional /
// filter-intra); the other units are read without a wait and may be stale or half-written,
// and no predicted pixel depends on them.  A predictor that starts reading a sample its mode
// did not read before must widen intra_needs first.

// Work-item encoding of the per-level item lists (host schedule -> k_level):
// bits 31..30 kind, 29..0 index (TB index; block index for inter-intra blends;
// block index << 4 | tile row << 2 | tile column for inter tiles).
#define AV1R_ITEM_TB 0u
#define AV1R_ITEM_INTER 1u
#define AV1R_ITEM_II 2u
#define AV1R_ITEM(kind, idx) (((uint32_t)(kind) << 30) | (uint32_t)(idx))
#define AV1R_ITEM_KIND(v) ((v) >> 30)
#define AV1R_ITEM_INDEX(v) ((v) & 0x3fffffffu)

// ---- debug timeline of the recon kernels (-DAV1R_TRACE; recon.hip) ----
#define AV1R_TRACE_W 16  // u64 per item in the debug timeline
// Debug timeline (AV1R_TRACE_FILE): lane 0 of each item stamps the 100 MHz real-time
// counter at entry, once the item record is in, after the prediction and at the end.
// Compiled in only with -DAV1R_TRACE (the stamps' waits constrain scheduling).
DEV void trace_put(unsigned long long* tr, int slot, unsigned long long v)
{
#ifdef AV1R_TRACE
    if (tr && (threadIdx.x & 63) == 0) tr[slot] = v;
#else
    (void)tr;
    (void)slot;
    (void)v;
#endif
}
DEV unsigned long long trace_now()
{
#ifdef AV1R_TRACE
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    return __builtin_amdgcn_s_memrealtime();
#else
    return 0;
#endif
}
// -DAV1R_TRACE_LITE (with AV1R_TRACE): the stamps wait for nothing and go to an LDS row per
// wave, copied to the timeline by trace_flush at the item's end -- the time a wave reaches
// each point of its instruction stream, without the drains of the full build
#ifdef AV1R_TRACE_LITE
DEV unsigned long long* lite_slots()
{
    __shared__ unsigned long long rows[4][AV1R_TRACE_W];
    return rows[(threadIdx.x >> 6) & 3];
}
#endif
DEV void trace_stamp(unsigned long long* tr, int slot)
{
#if defined(AV1R_TRACE) && defined(AV1R_TRACE_LITE)
    if (tr && (threadIdx.x & 63) == 0) lite_slots()[slot] = __builtin_amdgcn_s_memrealtime();
#elif defined(AV1R_TRACE)
    if (tr && (threadIdx.x & 63) == 0) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        tr[slot] = __builtin_amdgcn_s_memrealtime();
    }
#else
    (void)tr;
    (void)slot;
#endif
}
DEV void trace_flush(unsigned long long* tr)
{
#if defined(AV1R_TRACE) && defined(AV1R_TRACE_LITE)
    if (tr && (threadIdx.x & 63) == 0)
        for (int q = 2; q < 14; q++)
            if (q != 6 && q != 7) {
                tr[q] = lite_slots()[q];
                lite_slots()[q] = 0;
            }
#else
    (void)tr;
#endif
}


