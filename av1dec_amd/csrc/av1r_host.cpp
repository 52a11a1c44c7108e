// av1r_host.cpp -- host runtime of the gfx950 reconstruction backend and its C-ABI.
//
// Replaces, below the parse/reconstruct seam, the reference decoder's
// Decoder::decodeFrame / decode_frame_wrapup / updateFrameStore / getOutput
// (decoder/Av1Decoder.cpp:111-211).  Per frame it
//   1. validates the batch (every index a kernel will follow is range-checked here),
//   2. derives the dependency schedule: each inter block's prediction and each
//      transform block becomes a work item whose level is 1 + the highest level of
//      the items that produced the pixels it reads (intra edges, CFL luma, inter-intra
//      edges, intra-block-copy source) -- the decode-order dependencies of
//      TransformBlock::decode / IntraPredict::predict_intra made explicit,
//   3. uploads batch + schedule with ONE async copy from pinned memory,
//   4. launches per level {k_inter, k_tb}, then k_lf (2 passes), k_cdef, k_lr on the
//      context's HIP stream, and updates the 8-slot device frame store.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "av1r_dev.h"

void launch_k_level(int kind, const KParams* kps, const uint32_t* tab, int n, unsigned items, unsigned long long* trace,
    uint32_t traceBase, hipStream_t s);
void launch_k_inter_all(const KParams* kps, const uint32_t* tab, int n, uint32_t gI, uint32_t gM, uint32_t gS, uint32_t nb,
    unsigned long long* trace, hipStream_t s);
void launch_k_lf(const KParams* kps, int n, int pass, int maxUnits, hipStream_t s);
void launch_k_cdef(const KParams* kps, int n, int maxMiCols, int maxMiRows, hipStream_t s);
void launch_k_lr(const KParams* kps, int n, int maxW, int maxH, hipStream_t s);
#ifdef AV1R_FUSED_STRIPE
void launch_k_stripe(const KParams* kps, int n, int maxW, int maxH, int runTiles, hipStream_t s);
#endif
void launch_k_copy_plane(const DevPlane& dst, const DevPlane& src, hipStream_t s);
void launch_k_fetch(void* dst, const void* src, size_t bytes, hipStream_t s);
void launch_k_mi(const KParams* kps, int n, uint32_t maxUnits, uint32_t maxBlocks, uint32_t maxTbs, hipStream_t s);
#ifdef AV1R_FLOW_DEBUG
uint32_t flow_debug_overlaps(uint32_t* pairs, int n, int reset);
#endif
int flow_grid(int device, int maxPer);
void launch_k_resid(int large, const KParams* kps, const uint32_t* tab, int n, unsigned groups, hipStream_t s);
void launch_k_flow(const KParams* kps, const void* groups, uint32_t nGroups, uint32_t* ctl, uint32_t* hostErr,
    uint32_t epoch, int grid, unsigned long long* trace, hipStream_t s);

namespace {

struct FrameBuf {
    uint8_t* base = nullptr;
    size_t bytes = 0;
    int refcnt = 0;
    uint64_t seq = 0;  // the owning context's frame sequence number of the launch that wrote it
    // the launch that wrote it: its metadata slot and that slot's generation (
    // a read-back ticket waits for exactly this launch, whatever the context did since)
    const struct Upload* wMeta = nullptr;
    uint64_t wGen = 0;
    DevFrame d;
};

struct Upload {
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;  // all work that reads this upload has finished
    bool pending = false;
    std::atomic<uint64_t> gen{0};  // meta: launches that have used this slot (read by packers)
    // packed-frame slots (AV1R_SLOT_META): done when the launch that used meta slot waitMeta
    // at generation waitGen is (that launch's own completion event, no event of this slot's)
    const Upload* waitMeta = nullptr;
    uint64_t waitGen = 0;
};

struct Level {
    // items [off, off + cnt): [0] inter tiles (k_inter); k_tb's [1] large items (inter-intra
    // blends, TBs with a side >= 32: a workgroup each) and [2] small TBs (one per wave).
    // Within [1] and [2] the inter TBs come last: k_flow takes the first fcnt (inter TBs
    // are finished by k_resid there)
    // List [0] ends with pl[0] medium then pl[1] small plain blocks (k_inter_m two per wave,
    // k_inter_s four per wave; see build_schedule).  List [2] starts with `tiny` items
    // (TinyItem, k_flow's tiny groups; flow-only frames with granules).
    uint32_t off[3] = {}, cnt[3] = {}, fcnt[3] = {};
    uint32_t pl[2] = {};
    uint32_t tiny = 0;
};

inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

}  // namespace

// A frame whose batch and schedule are resident in device memory.
struct Prepared {
    uint8_t* dev = nullptr;  // owned buffer (prepared frames) or ring slot (streaming)
    size_t cap = 0;
    bool owned = false;
    av1r_frame_hdr hdr;
    KParams base;  // batch pointers into dev
    const WorkItem* dItems = nullptr;
    std::vector<Level> levels;
    bool flowOk = false;  // k_flow can run it: no inter tile after level 0 (intra block copy)
    bool levelsOk = true; // the level launches can run it (false: a flow-only schedule)
    uint32_t nResidS = 0, nResidL = 0;  // k_resid workgroups (64 4x4 TBs or 16 TBs / 1 TB each)
    size_t resElems = 0;                // int16 residual tiles of the frame
    bool usedRef[8] = {};
    uint64_t bytes = 0;    // the packed layout (incl. the device-filled mode-info grid)
    size_t upBytes = 0;    // its uploaded prefix
    bool offsets = false;  // packed in host memory: base pointers are offsets into the upload
};

// A frame validated, scheduled and packed into (pinned) host memory by av1r_pack, on any
// thread, ahead of its launch; av1r_decode_packed_batch uploads and decodes it.
struct av1r_packed {
    Prepared P;
    uint8_t* host = nullptr;
    size_t cap = 0;
    bool pinned = false;
    hipEvent_t copied = nullptr;  // the upload of this buffer (its host memory is in use until then)
    bool copyPending = false;
    // ... or the completion of the launch that read the upload: its meta slot and
    // that slot's generation then (see Upload::waitMeta)
    const struct Upload* waitMeta = nullptr;
    uint64_t waitGen = 0;
};

// One asynchronous read-back of a shown frame (av1r_get_output_async): the frame stays
// referenced (out of the pool) until the ticket is waited for.  The copies are issued on the
// context's output stream only once the frame's kernels have completed (`ready` observed
// by av1r_output_query / _wait), so the output stream never carries a cross-stream wait.
struct av1r_output_ticket {
    av1r_ctx* c = nullptr;
    FrameBuf* f = nullptr;
    uint8_t* dst[3] = {};
    int ds[3] = {};
    hipEvent_t ready = nullptr, done = nullptr;
    int state = 0;  // 0 the frame's kernels may still run, 1 copies issued, 2 landed
    bool live = false;
    bool sq = false;  // this read-back's landing is seen by the stream going idle
    // the frame is done when this launch is (the last launch on the frame's
    // stream, through its metadata slot and generation) instead of by `ready`
    const Upload* readyMeta = nullptr;
    uint64_t readyGen = 0;
};

struct av1r_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::vector<FrameBuf*> pool;
    FrameBuf* slots[8] = {};
    std::deque<FrameBuf*> outq;
    FrameBuf* stage[4] = {};
    bool keepStages = true;
    Upload up[2];
    int upIdx = 0;
#ifndef AV1R_RING
#define AV1R_RING 3
#endif
    static constexpr int kPackRing = AV1R_RING;  // device slots of packed uploads (av1r_decode_packed_batch)
    Upload pk[kPackRing];
    int pkIdx = 0;
    hipEvent_t pkReady = nullptr;  // the packed uploads of a batch (lead's copy stream) have landed
    // per-launch metadata (KParams, tables, flow groups): a ring, uploaded on a copy stream
    // of its own so that the copy of batch N + 1 overlaps the kernels of batch N
    static constexpr int kMetaRing = AV1R_RING;
    Upload meta[kMetaRing];
    const Upload* lastMeta = nullptr;  // the meta slot of this context's last launch (launch_jobs)
    int metaIdx = 0;
    hipStream_t copyStream = nullptr;
    // asynchronous frame delivery (av1r_get_output_async): the read-back copies' own stream
    // (created at the first such call) and every ticket ever allocated (free ones reused)
    hipStream_t outStream = nullptr;
    std::vector<av1r_output_ticket*> tickets;
    // av1r_set_output_prefetch: every shown frame's read-back starts at once into a pinned
    // staging buffer of the context (frames move from outq to `staged`, the older ones);
    // av1r_get_output then waits for that copy only and copies the rows out on the host
    struct Staged {
        av1r_output_ticket* t;
        uint8_t* buf;
        size_t cap;
        int w, h;
    };
    bool prefetch = false;
    std::deque<Staged> staged;
    std::vector<std::pair<uint8_t*, size_t>> stageFree;
    hipEvent_t sync = nullptr;  // cross-context ordering of batched launches
    // this context's latest work was launched on joinLead's stream (a batch it was a member
    // of) and nothing has been enqueued on its own stream since; ctx_join() orders its own
    // stream after that work before anything else uses it
    av1r_ctx* joinLead = nullptr;
    hipEvent_t joinEv = nullptr;
    // debug timeline of every recon work item (env AV1R_TRACE_FILE): 8 x u64 per item
    FILE* traceFile = nullptr;
    unsigned long long* traceDev = nullptr;
    size_t traceCap = 0;
    std::string err;
    // schedule scratch: per 4x4 unit and plane, its level (the item that last wrote it), its
    // owner node and whether it is on its owner's bottom row / right column (one 8-byte
    // record per unit: the three lookups of a unit share a cache line)
    struct MapUnit {
        int32_t owner;
        int16_t lvl;
        uint8_t emit;
        uint8_t pad;
    };
    std::vector<MapUnit> umap[3];
    int mapW[3] = {}, mapH[3] = {};
    std::vector<std::vector<uint32_t>> lvP, lvB, lvT;  // inter tiles, inter-intra blends, TBs per level
    std::vector<WorkItem> items;  // transform blocks and inter-intra blends
    // pack_frame, from its size pass for its packing pass: whether any TB has a level that
    // needs more than 6 signed bits, and then per TB its width (AV1R_TBD_WIDE) and a wide
    // TB's offset in the 32-bit array
    bool anyWide = false, wideKnown = false;  // (wideKnown: validate's fast pass classified)
    std::vector<uint32_t> tbCoefOff;
    std::vector<uint8_t> tbWide;
    size_t nCoef32 = 0;
    std::vector<uint32_t> tiles;  // inter tiles (codes): Level::off[0] indexes them
    std::vector<Level> levels;
    // k_flow dependencies: per 4x4 unit the node (TB / inter-intra item, decode order) that
    // last wrote it (-1: nothing, or an inter tile of the preceding launch); per node its
    // dependency nodes (CSR); then, in item order, the dependencies' item positions
    std::vector<uint32_t> nodeDepStart;
    std::vector<int32_t> nodeDeps, nodeOfTb, nodeOfBlk, nodePos;
    // critical-path order (flow-only frames, build_schedule): per node its level and the
    // producers of the edge units it reads through granules (not in nodeDeps), as CSR; the
    // height (longest chain of consumers below a node)
    std::vector<int32_t> nodeLvl, edgeDeps, nodeHeight;
    std::vector<uint32_t> edgeStart;
    std::vector<uint32_t> deps;
    bool flowOk = false;
    bool levelsOk = true;  // the level schedule was built too (not a flow-only schedule)
    bool usedRef[8] = {};  // validate(): references the mode-info grid uses
    // k_flow edge granules (KParams::gran_h / gran_v): per 4x4 unit whether it is on the
    // bottom row / right column of its owner (the units whose granules the owner stores);
    // per node 12 mask words (4 per plane: the above and left runs' units written by an
    // item of the launch); granOk = every such unit a consumer reads has its granule
    std::vector<uint32_t> nodeMask;
    bool granOk = false;
    uint64_t* granDev = nullptr;
    size_t granCap = 0;  // bytes
    // k_resid: per TB its residual tile offset (int16 elements, ~0u: none / added in place),
    // the small and large TB lists, the tiles' total size
    std::vector<uint32_t> tbRes, residS, residL, residT, residE, residM;
    uint32_t nResidM = 0;  // k_resid_l workgroups of two TBs with both sides <= 32 (32 lanes each), heading residL
    uint32_t nResidT = 0;  // k_resid_s workgroups of 4x4 TBs (the head of residS)
    uint32_t nResidE = 0;  // then workgroups of 32 TBs with both sides <= 8 (8 lanes each)
    size_t resElems = 0;
    // split submission (frame_begin / submit_tile / frame_end)
    bool inFrame = false;
    std::vector<uint8_t> fHdr;
    std::vector<av1r_mi> fMi;
    std::vector<int8_t> fCdef;
    std::vector<av1r_lr_unit> fLr;
    std::vector<av1r_block> fBlocks;
    std::vector<av1r_tb> fTbs;
    std::vector<uint32_t> fCoefs;
    std::vector<uint8_t> fPal;
    // timing: one set of 5 stage-boundary events per frame since the last summary
    bool timing = false;
    // [0] start, [1] recon end, [2] LF end, [3] CDEF end, [4] LR end; k_flow mode also
    // [5] after k_inter, [6] after k_resid (zero-length spans in level mode)
    hipEvent_t ev[7] = {};
    std::vector<std::array<hipEvent_t, 7>> evPool;
    std::vector<int> evFrames;  // frames covered by each event set (batched launches)
    size_t evUsed = 0;
    int nLevelsLast = 0;
    // stats of the last frame
    uint64_t lastUploadBytes = 0;
    bool skipSlotCheck = false;  // av1r_check_batch: no frame store to resolve against
    bool discardOutput = false;  // bench: shown frames are not queued for read-back
    Prepared streamP;
    std::vector<Prepared*> prepared;
    int schedule = -1;  // av1r_set_schedule: -1 default (AV1R_FLOW), 0 level launches, 1 k_flow
    int16_t* resDev = nullptr;  // k_flow mode: the frame's residual tiles (k_resid)
    size_t resCap = 0;
    uint32_t flowSpins = 0;     // av1r_set_flow_spins (0: FLOW_SPINS)
    int flowPerCU = 8;          // k_flow workgroups per CU of this context's launches (capped by occupancy)
    // a deep frame launched alone on this context's own stream (batched entry points): its
    // completion; av1r_busy reports whether it is still running
    hipEvent_t soloDone = nullptr;
    bool soloPending = false;
    // device-error bookkeeping (under g_recMu): frame sequence numbers of this context's
    // frames whose launch reported a k_flow timeout, those not yet returned by
    // av1r_synchronize, and the sequence numbers of key frames refreshing every slot (a
    // failure taints every later frame of the stream up to the next such key frame)
    uint64_t seq = 0, lastSeq = 0;
    std::vector<uint64_t> failed, keySeqs;
    size_t failedReported = 0;
};

// A launch that ran k_flow: its pinned error word (the kernel writes it when a wait
// times out), an event after the launch's last kernel, and the frames it produced as
// (context, frame sequence number).  When the event has completed the record is
// harvested: a set error word marks those frames failed in EVERY member context.
struct LaunchRec {
    uint32_t* err = nullptr;
    hipEvent_t done = nullptr;
    const struct Upload* meta = nullptr;  // completion = this launch's meta slot
    uint64_t gen = 0;
    std::vector<std::pair<av1r_ctx*, uint64_t>> members;
};
static std::mutex g_recMu;
static std::vector<LaunchRec*> g_recPending, g_recFree;
// packed frames (av1r_pack) released by their launches, for reuse by any packing thread
static std::mutex g_packMu;
static std::vector<av1r_packed*> g_packFree;
static std::vector<av1r_packed*> g_packAll;  // every packed buffer ever allocated (under g_packMu)

// Completion of a launch through its own meta slot (the one event every launch records on
// its stream after its last kernel) instead of more events recorded after it: a launch
// recorded one per packed-frame slot, one per packed buffer and one for its status record
// -- each a marker packet in the compute stream's hardware queue.  Without them (round 4)
// the headline rose 6 100 -> 6 370 frames/s.
// The meta slot's generation counts its launches: once it has moved on, the launch waited
// for was synchronized before the slot's reuse.
static bool meta_done(const Upload* m, uint64_t gen)
{
    return m->gen.load(std::memory_order_acquire) != gen || hipEventQuery(m->done) == hipSuccess;
}
static void meta_wait(const Upload* m, uint64_t gen)
{
    if (m->gen.load(std::memory_order_acquire) == gen) (void)hipEventSynchronize(m->done);
}

// collect completed launch records (wait: block on each pending one first)
static void harvest(bool wait)
{
    std::lock_guard<std::mutex> lock(g_recMu);
    for (size_t i = 0; i < g_recPending.size();) {
        LaunchRec* r = g_recPending[i];
        if (r->meta) {
            if (wait) meta_wait(r->meta, r->gen);
            if (!meta_done(r->meta, r->gen)) {
                i++;
                continue;
            }
        } else {
            if (wait) (void)hipEventSynchronize(r->done);
            if (hipEventQuery(r->done) != hipSuccess) {
                i++;
                continue;
            }
        }
        if (const uint32_t e = *r->err) {
            for (auto& m : r->members) {
                m.first->failed.push_back(m.second);
                m.first->err = e == 2 ? "k_flow: an edge granule wait timed out (frame output invalid)"
                                      : "k_flow: a dependency wait timed out (frame output invalid)";
            }
            *r->err = 0;
        }
        r->members.clear();
        g_recFree.push_back(r);
        g_recPending[i] = g_recPending.back();
        g_recPending.pop_back();
    }
}

// whether frame `seq` of context c is corrupt: some failed frame b <= seq of its stream
// with no key frame refreshing every slot in (b, seq]  (caller holds g_recMu)
static bool frame_failed(const av1r_ctx* c, uint64_t seq)
{
    for (uint64_t b : c->failed) {
        if (b > seq) continue;
        bool healed = false;
        for (uint64_t k : c->keySeqs) healed |= k > b && k <= seq;
        if (!healed) return true;
    }
    return false;
}

// live contexts (a destroyed batch lead must not stay another context's joinLead)
static std::mutex g_ctxMu;
static std::vector<av1r_ctx*> g_ctxs;

// Lazy cross-stream ordering of batch members (av1r_decode_prepared_batch): called before
// anything enqueues on, or waits for, the context's own stream.
static int stage_outputs(av1r_ctx* c);

static void ctx_join(av1r_ctx* c)
{
    if (!c || !c->joinLead) return;
    (void)hipEventRecord(c->joinEv, c->joinLead->stream);
    (void)hipStreamWaitEvent(c->stream, c->joinEv, 0);
    c->joinLead = nullptr;
}

static int fail(av1r_ctx* c, int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}
#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) return fail(c, AV1R_E_DEVICE, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

static void frame_unref(av1r_ctx* c, FrameBuf* f)
{
    if (f && f->refcnt > 0) f->refcnt--;
}
static void frame_ref(FrameBuf* f)
{
    if (f) f->refcnt++;
}

// A frame's planes in one allocation: rows padded to 128 + 64 pixels (256-byte aligned
// strides), 64 + 128-aligned rows, each plane 256-byte aligned (av1r_frame_layout)
struct FrameGeom {
    int stride[3];
    size_t off[3];
    size_t bytes;  // the allocation
    size_t span;   // plane 0's first byte to the last visible byte of plane 2
};
static FrameGeom frame_geom(int width, int height)
{
    FrameGeom g;
    const int aw = ((width + 127) & ~127) + 64, ah = ((height + 127) & ~127) + 64;
    g.stride[0] = (int)align256(aw);
    g.stride[1] = g.stride[2] = (int)align256(aw / 2);
    const size_t ySz = (size_t)g.stride[0] * ah, cSz = (size_t)g.stride[1] * (ah / 2);
    g.off[0] = 0;
    g.off[1] = align256(ySz);
    g.off[2] = g.off[1] + align256(cSz);
    g.bytes = g.off[2] + align256(cSz);
    g.span = g.off[2] + (size_t)g.stride[2] * ((height >> 1) - 1) + (width >> 1);
    return g;
}

static FrameBuf* frame_get(av1r_ctx* c, int width, int height)
{
    const FrameGeom g = frame_geom(width, height);
    const int strideY = g.stride[0], strideC = g.stride[1];
    const size_t need = g.bytes;
    FrameBuf* f = nullptr;
    for (FrameBuf* p : c->pool)
        if (p->refcnt == 0 && p->bytes >= need) {
            f = p;
            break;
        }
    if (!f) {
        f = new FrameBuf;
        if (hipMalloc(&f->base, need) != hipSuccess) {
            delete f;
            return nullptr;
        }
        ctx_join(c);
        (void)hipMemsetAsync(f->base, 0, need, c->stream);
        f->bytes = need;
        c->pool.push_back(f);
    }
    f->refcnt = 1;
    f->d.width = width;
    f->d.height = height;
    f->d.pl[0] = {f->base + g.off[0], strideY, width, height};
    f->d.pl[1] = {f->base + g.off[1], strideC, width >> 1, height >> 1};
    f->d.pl[2] = {f->base + g.off[2], strideC, width >> 1, height >> 1};
    return f;
}

// ------------------------------------------------------------------------------------
// batch validation: everything a kernel dereferences is checked here
// ------------------------------------------------------------------------------------
// KParams' section pointers in their packing order (pack_frame).  The packed path keeps
// them as offsets into the frame's buffer and rebases every one at launch (job_begin): one
// list for the packing check and the rebase, so that no section is placed and left
// unrebased (round 6: a residual-tile section added to the packing and not to the rebase
// faulted on the device)
#define AV1R_KP_SECTIONS(X) X(hdr) X(blocks) X(bext) X(tbs) X(coefs) X(coefs16) X(palette) X(cdef_idx) X(lr) X(items) \
    X(tiles) X(deps) X(tb_res) X(resid_s) X(resid_l) X(done) X(mi)

static int validate(av1r_ctx* c, const av1r_frame_batch* b)
{
    const av1r_frame_hdr* h = b->hdr;
    if (h->bitdepth != 8 || h->subx != 1 || h->suby != 1)
        return fail(c, AV1R_E_UNSUPPORTED, "only 8-bit 4:2:0 is supported (reference README)");
    if ((h->frame_width & 1) || (h->frame_height & 1) || h->frame_width <= 0 || h->frame_height <= 0 || h->frame_width > 16384 || h->frame_height > 16384)
        return fail(c, AV1R_E_UNSUPPORTED, "frame size %dx%d not supported", h->frame_width, h->frame_height);
    if (h->mi_cols != 2 * ((h->frame_width + 7) >> 3) || h->mi_rows != 2 * ((h->frame_height + 7) >> 3))
        return fail(c, AV1R_E_INVALID, "MiCols/MiRows inconsistent with the frame size");
    int sb4 = h->sb128 ? 32 : 16;
    if (h->mi_stride < ((h->mi_cols + sb4 - 1) / sb4) * sb4 || h->mi_rows_alloc < ((h->mi_rows + sb4 - 1) / sb4) * sb4)
        return fail(c, AV1R_E_INVALID, "mode-info grid smaller than the SB-aligned frame");
    if (!b->cdef_idx) return fail(c, AV1R_E_INVALID, "missing cdef grid");
    if (h->cdef_rows != (h->mi_rows + 15) / 16 || h->cdef_cols != (h->mi_cols + 15) / 16)
        return fail(c, AV1R_E_INVALID, "cdef grid dims");
    for (int i = 0; i < h->cdef_rows * h->cdef_cols; i++)
        if (b->cdef_idx[i] < -1 || b->cdef_idx[i] > 7) return fail(c, AV1R_E_INVALID, "cdef_idx out of range");
    const int aw4 = h->mi_stride, ah4 = h->mi_rows_alloc;
    // the blocks' reference frames (and the slots they resolve to): one branch-free pass
    // accumulating the violations; the block loop below names the first one.  (The mode-info
    // grid is not read: the device derives it from the blocks and transform blocks.)
    bool* usedRef = c->usedRef;
    memset(c->usedRef, 0, sizeof(c->usedRef));
    uint32_t bad = 0, refs = 0;
    for (uint32_t i = 0; i < b->n_blocks; i++) {
        const av1r_block& k = b->blocks[i];
        bad |= ((uint8_t)(k.ref_frame[0] + 1) > 8) | ((uint8_t)(k.ref_frame[1] + 1) > 8) | ((k.filt & 15) > 3) | ((k.filt >> 4) > 3);
        refs |= (1u << ((k.ref_frame[0] + 1) & 15)) | (1u << ((k.ref_frame[1] + 1) & 15));
    }
    for (uint32_t i = 0; bad && i < b->n_blocks; i++) {
        const av1r_block& k = b->blocks[i];
        for (int l = 0; l < 2; l++)
            if (k.ref_frame[l] < -1 || k.ref_frame[l] > 7) return fail(c, AV1R_E_INVALID, "block %u ref_frame", i);
        if ((k.filt & 15) > 3 || (k.filt >> 4) > 3) return fail(c, AV1R_E_INVALID, "block %u interp filter", i);
    }
    for (int r = 1; r < 8; r++) usedRef[r] = (refs >> (r + 1)) & 1;
    for (int r = 1; r < 8 && !c->skipSlotCheck; r++) {
        if (!usedRef[r]) continue;
        int slot = h->ref_frame_idx[r - 1];
        if (slot < 0 || slot > 7 || !c->slots[slot])
            return fail(c, AV1R_E_INVALID, "reference %d maps to an empty slot", r);
    }
    if (b->n_blocks >= (1u << 26) || b->n_tbs >= (1u << 30))
        return fail(c, AV1R_E_UNSUPPORTED, "too many blocks / transform blocks in one frame");
    // the checks below in branch-free passes first (every violation ORed into one word);
    // only a batch that fails one walks the detailed loops, which name the first violation
    {
        uint32_t badB = 0, badT = 0;
        bool anyPal = false;
        for (uint32_t i = 0; i < b->n_blocks; i++) {
            const av1r_block& k = b->blocks[i];
            const uint32_t sz = k.mi_size < AV1R_BLOCK_SIZES ? k.mi_size : 0;
            const bool inter = k.flags & AV1R_BLK_INTER;
            badB |= (k.mi_size >= AV1R_BLOCK_SIZES) | ((uint32_t)k.mi_row + av1r_num4x4h[sz] > (uint32_t)ah4) |
                    ((uint32_t)k.mi_col + av1r_num4x4w[sz] > (uint32_t)aw4) | ((uint64_t)k.first_tb + k.n_tbs > b->n_tbs) |
                    (k.palette_size_y > 8) | (k.palette_size_uv > 8);
            anyPal |= (k.palette_size_y | k.palette_size_uv) != 0;
            const uint32_t badI = (k.motion_mode > 2) | (k.compound_type > 4) | (k.interintra_mode > 3) |
                                  ((k.compound_type == AV1R_COMPOUND_WEDGE) & ((k.wedge_index > 15) | !av1r_wedge_bits[sz])) |
                                  (((k.flags & AV1R_BLK_INTERINTRA) != 0) & ((k.mi_size < AV1R_BLOCK_8X8) | (k.mi_size > AV1R_BLOCK_32X32)));
            const uint32_t badA = (k.y_mode > AV1R_PAETH_PRED) | (((k.flags & AV1R_BLK_HAS_CHROMA) != 0) & (k.uv_mode > AV1R_UV_CFL_PRED)) |
                                  (((k.flags & AV1R_BLK_FILTER_INTRA) != 0) & (k.filter_intra_mode > 4));
            badB |= inter ? badI : badA;
            // the device reaches an inter-intra block's TB range and a local warp through
            // palette_off (DevBlock, pack_frame): those flags only on inter blocks without a
            // palette, and INTERINTRA exactly when build_schedule makes the block an
            // inter-intra item (inter with ref_frame[1] == INTRA_FRAME)
            const bool ext = (k.flags & (AV1R_BLK_LOCAL_VALID | AV1R_BLK_INTERINTRA)) != 0;
            const bool ii = inter && k.ref_frame[1] == AV1R_INTRA_FRAME;
            badB |= (ext & (!inter | ((k.palette_size_y | k.palette_size_uv) != 0))) |
                    (ii != ((k.flags & AV1R_BLK_INTERINTRA) != 0));
        }
        for (uint32_t i = 0; i < b->n_tbs; i++) {
            const av1r_tb& t = b->tbs[i];
            const uint32_t tx = t.tx_size < AV1R_TX_SIZES ? t.tx_size : 0;
            const int sub = t.plane ? 1 : 0;
            badT |= (t.block >= b->n_blocks) | (t.plane > 2) | (t.tx_size >= AV1R_TX_SIZES) | (t.tx_type > 15) |
                    (t.x + av1r_tx_w[tx] > ((aw4 * 4) >> sub) + 64) | (t.y + av1r_tx_h[tx] > ((ah4 * 4) >> sub) + 64) |
                    ((uint64_t)t.coef_off + t.coef_cnt > b->n_coefs);
        }
        uint32_t badC = 0;
        // (with the positions, each TB's coefficient width for pack_frame: a level outside 6
        // signed bits makes (c + 0x8000) >> 16 non-zero)
        c->tbWide.resize(b->n_tbs);
        uint32_t anyWide = 0;
        if (!badT)
            for (uint32_t i = 0; i < b->n_tbs; i++) {
                const av1r_tb& t = b->tbs[i];
                const int log2Area = std::min<int>(av1r_tx_w_log2[t.tx_size], 5) + std::min<int>(av1r_tx_h_log2[t.tx_size], 5);
                uint32_t acc = 0, wide = 0;
                const uint32_t* cf = b->coefs + t.coef_off;
                const uint32_t n = t.coef_cnt;
                if ((uint64_t)t.coef_off + 16 <= b->n_coefs) {
                    // the first 16 (most TBs have fewer) masked, without a data-dependent
                    // branch: a short loop per TB mispredicted its exit once per TB
                    for (uint32_t q = 0; q < 16; q++) {
                        const uint32_t m = q < n ? ~0u : 0u;
                        acc |= cf[q] & m;
                        wide |= ((cf[q] + 0x8000u) >> 16) & m;
                    }
                    for (uint32_t q = 16; q < n; q++) acc |= cf[q], wide |= (cf[q] + 0x8000u) >> 16;
                } else {
                    for (uint32_t q = 0; q < n; q++) acc |= cf[q], wide |= (cf[q] + 0x8000u) >> 16;
                }
                badC |= (acc & 1023u) >> log2Area;
                c->tbWide[i] = wide != 0;
                anyWide |= wide;
            }
        c->anyWide = anyWide != 0;
        c->wideKnown = !badT;
        // palette blocks (rare): their records, then the map window of every transform block
        // whose OWN block (t.block: what build_schedule and the device's tb_predict follow) is
        // an intra palette block -- wherever that TB sits in the TB array
        for (uint32_t i = 0; anyPal && !badB && i < b->n_blocks; i++) {
            const av1r_block& k = b->blocks[i];
            if (!(k.palette_size_y || k.palette_size_uv)) continue;
            if ((uint64_t)k.palette_off + AV1R_PALETTE_HDR > b->n_palette) badB = 1;
            else {
                const uint8_t* ph = b->palette + k.palette_off;
                if ((uint64_t)k.palette_off + AV1R_PALETTE_HDR + ph[0] * ph[1] + ph[2] * ph[3] > b->n_palette) badB = 1;
            }
        }
        for (uint32_t ti = 0; anyPal && !badB && !badT && ti < b->n_tbs; ti++) {
            const av1r_tb& t = b->tbs[ti];
            const av1r_block& k = b->blocks[t.block];
            if ((k.flags & AV1R_BLK_INTER) || !(t.plane ? k.palette_size_uv : k.palette_size_y)) continue;
            const uint8_t* ph = b->palette + k.palette_off;
            const int sub = t.plane ? 1 : 0;
            const int bx = t.x - (k.mi_col >> sub) * 4, by = t.y - (k.mi_row >> sub) * 4;
            const int mw = t.plane ? ph[2] : ph[0], mh = t.plane ? ph[3] : ph[1];
            badT |= (bx < 0) | (by < 0) | (bx + av1r_tx_w[t.tx_size] > mw) | (by + av1r_tx_h[t.tx_size] > mh);
        }
        if (!badB && !badT && !badC) goto lr_check;
    }
    for (uint32_t i = 0; i < b->n_blocks; i++) {
        const av1r_block& k = b->blocks[i];
        if (k.mi_size >= AV1R_BLOCK_SIZES || k.mi_row >= ah4 || k.mi_col >= aw4
            || k.mi_row + av1r_num4x4h[k.mi_size] > ah4 || k.mi_col + av1r_num4x4w[k.mi_size] > aw4)
            return fail(c, AV1R_E_INVALID, "block %u geometry", i);
        if ((uint64_t)k.first_tb + k.n_tbs > b->n_tbs) return fail(c, AV1R_E_INVALID, "block %u tb range", i);
        if (k.palette_size_y > 8 || k.palette_size_uv > 8) return fail(c, AV1R_E_INVALID, "palette size");
        if (k.palette_size_y || k.palette_size_uv) {
            if ((uint64_t)k.palette_off + AV1R_PALETTE_HDR > b->n_palette) return fail(c, AV1R_E_INVALID, "palette offset");
            const uint8_t* ph = b->palette + k.palette_off;
            if ((uint64_t)k.palette_off + AV1R_PALETTE_HDR + ph[0] * ph[1] + ph[2] * ph[3] > b->n_palette)
                return fail(c, AV1R_E_INVALID, "palette map size");
        }
        if (k.flags & AV1R_BLK_INTER) {
            if (k.motion_mode > 2 || k.compound_type > 4 || k.interintra_mode > 3
                || (k.compound_type == AV1R_COMPOUND_WEDGE && k.wedge_index > 15))
                return fail(c, AV1R_E_INVALID, "block %u inter params", i);
            if (k.compound_type == AV1R_COMPOUND_WEDGE && !av1r_wedge_bits[k.mi_size])
                return fail(c, AV1R_E_INVALID, "wedge on a block size without wedges");
            if (k.flags & AV1R_BLK_INTERINTRA)
                if (k.mi_size < AV1R_BLOCK_8X8 || k.mi_size > AV1R_BLOCK_32X32) return fail(c, AV1R_E_INVALID, "interintra size");
            if ((k.ref_frame[1] == AV1R_INTRA_FRAME) != ((k.flags & AV1R_BLK_INTERINTRA) != 0))
                return fail(c, AV1R_E_INVALID, "block %u: INTERINTRA flag disagrees with ref_frame[1]", i);
        }
        if ((k.flags & (AV1R_BLK_LOCAL_VALID | AV1R_BLK_INTERINTRA))
            && (!(k.flags & AV1R_BLK_INTER) || k.palette_size_y || k.palette_size_uv))
            return fail(c, AV1R_E_INVALID, "block %u: warp / inter-intra flags on an intra or palette block", i);
        if (!(k.flags & AV1R_BLK_INTER)) {
            if (k.y_mode > AV1R_PAETH_PRED || ((k.flags & AV1R_BLK_HAS_CHROMA) && k.uv_mode > AV1R_UV_CFL_PRED)
                || ((k.flags & AV1R_BLK_FILTER_INTRA) && k.filter_intra_mode > 4))
                return fail(c, AV1R_E_INVALID, "block %u intra modes", i);
        }
    }
    for (uint32_t i = 0; i < b->n_tbs; i++) {
        const av1r_tb& t = b->tbs[i];
        if (t.block >= b->n_blocks || t.plane > 2 || t.tx_size >= AV1R_TX_SIZES || t.tx_type > 15)
            return fail(c, AV1R_E_INVALID, "tb %u fields", i);
        int sub = t.plane ? 1 : 0;
        if (t.x + av1r_tx_w[t.tx_size] > ((aw4 * 4) >> sub) + 64 || t.y + av1r_tx_h[t.tx_size] > ((ah4 * 4) >> sub) + 64)
            return fail(c, AV1R_E_INVALID, "tb %u outside the frame", i);
        if ((uint64_t)t.coef_off + t.coef_cnt > b->n_coefs) return fail(c, AV1R_E_INVALID, "tb %u coefficients", i);
        // positions < area = min(w,32) * min(h,32), a power of two: no position has a bit at
        // or above log2(area) set, so one OR over the TB's coefficients decides (vectorised)
        const int log2Area = std::min<int>(av1r_tx_w_log2[t.tx_size], 5) + std::min<int>(av1r_tx_h_log2[t.tx_size], 5);
        uint32_t acc = 0;
        const uint32_t* cf = b->coefs + t.coef_off;
        for (int q = 0; q < t.coef_cnt; q++) acc |= cf[q];
        if ((acc & 1023u) >> log2Area) return fail(c, AV1R_E_INVALID, "tb %u coefficient position", i);
        const av1r_block& k = b->blocks[t.block];
        if (!(k.flags & AV1R_BLK_INTER) && (t.plane ? k.palette_size_uv : k.palette_size_y)) {
            const uint8_t* ph = b->palette + k.palette_off;
            int bx = t.x - (k.mi_col >> sub) * 4, by = t.y - (k.mi_row >> sub) * 4;
            int mw = t.plane ? ph[2] : ph[0], mh = t.plane ? ph[3] : ph[1];
            if (bx < 0 || by < 0 || bx + av1r_tx_w[t.tx_size] > mw || by + av1r_tx_h[t.tx_size] > mh)
                return fail(c, AV1R_E_INVALID, "tb %u palette map window", i);
        }
    }
lr_check:
    if (h->uses_lr) {
        for (int p = 0; p < 3; p++) {
            if (h->lr_type[p] == AV1R_RESTORE_NONE) continue;
            int us = h->lr_unit_size[p];
            if (us != 32 && us != 64 && us != 128 && us != 256) return fail(c, AV1R_E_INVALID, "lr unit size");
            if ((int64_t)h->lr_unit_off[p] + (int64_t)h->lr_unit_rows[p] * h->lr_unit_cols[p] > b->n_lr_units || h->lr_unit_rows[p] < 1 || h->lr_unit_cols[p] < 1)
                return fail(c, AV1R_E_INVALID, "lr units");
            for (int u = 0; u < h->lr_unit_rows[p] * h->lr_unit_cols[p]; u++)
                if (b->lr_units[h->lr_unit_off[p] + u].sgr_set > 15 || b->lr_units[h->lr_unit_off[p] + u].type > 2)
                    return fail(c, AV1R_E_INVALID, "lr unit params");
        }
    }
    return AV1R_OK;
}

// ------------------------------------------------------------------------------------
// av1r_pack profile (AV1R_PACK_PROF=1): nanoseconds per phase, summed over every thread
// ------------------------------------------------------------------------------------
enum { PP_VALIDATE, PP_SCHED_INIT, PP_SCHED_BLOCKS, PP_SCHED_ITEMS, PP_SCHED_DEPS, PP_COPY, PP_N };
static std::atomic<uint64_t> g_packNs[PP_N + 1];  // [PP_N]: packed frames
static const bool g_packProf = getenv("AV1R_PACK_PROF") && atoi(getenv("AV1R_PACK_PROF")) != 0;
struct PackClock {
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(int phase)
    {
        if (!g_packProf) return;
        const auto n = std::chrono::steady_clock::now();
        g_packNs[phase] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(n - t).count();
        t = n;
    }
};

// the lean small-intra path of k_flow (intra_fast.h); av1r_set_fast_intra(0): the generic
// path (A/B)
static std::atomic<int> g_fastIntra{1};

// ------------------------------------------------------------------------------------
// dependency levels
// ------------------------------------------------------------------------------------
// flowOnly: the frame will run on k_flow (av1r_pack; no intra block copy), so inter TBs
// outside inter-intra blocks -- finished by k_resid before k_flow -- get no node, item or
// level: only the level launches need them.  c->levelsOk says whether the level schedule
// was built too.
// The pixels an intra prediction actually uses (IntraPredict::predict_intra,
// IntraPredict.cpp:563-631, and the predictors it calls): the above-right run
// (x + w .. x + 2w - 1) only by a directional prediction at an angle below 90 (the
// zone-1 predictor, :379-483 with pAngle < 90, and its edge filter / upsampling over
// w + h samples); the below-left run only by one above 180 (zone 3).  DC, V, H, smooth,
// Paeth, CFL, filter-intra and the inter-intra modes (II_DC / V / H / SMOOTH) read at most
// w samples above and h on the left.  A TB's dependencies (and granule masks) cover only
// what its mode reads: the device gathers the rest of the run without waiting, and those
// samples never reach a predicted pixel.  angle: -1 for a non-directional prediction.
static int intra_angle(const av1r_block& blk, int p)
{
    if (p == 0 && (blk.flags & AV1R_BLK_FILTER_INTRA)) return -1;
    const int mode = p ? blk.uv_mode : blk.y_mode;  // (UV_CFL_PRED: not directional)
    if (mode < AV1R_V_PRED || mode > AV1R_D67_PRED) return -1;
    return av1r_mode_to_angle[mode] + (p ? blk.angle_delta_uv : blk.angle_delta_y) * 3;
}
// Which of the edge runs the prediction uses (bit 0 the above run, bit 1 the left run,
// bit 2 the corner pixel (x - 1, y - 1)): V reads only the row above and H only the column
// on the left (the other one stands in when a side is missing, :571-590), zone 1 the row and
// the corner (its edge filter / upsampling reach index -1), zone 3 the column and the
// corner; DC, smooth and CFL no corner; Paeth, zone 2 and filter-intra everything.
static int intra_needs(const av1r_block& blk, int p, bool hA, bool hL)
{
    const int mode = p ? blk.uv_mode : blk.y_mode;
    if ((p == 0 && (blk.flags & AV1R_BLK_FILTER_INTRA)) || mode == AV1R_PAETH_PRED) return 7;
    const int ang = intra_angle(blk, p);
    if (ang < 0) return 3;
    if (ang == 90) return hA ? 1 : 3;
    if (ang == 180) return hL ? 2 : 3;
    if (ang < 90) return hA ? 5 : 7;
    if (ang > 180) return hL ? 6 : 7;
    return 7;
}

// k_flow's small-item groups: four items (one per wave) on a thin level, 8 (two per wave,
// run one after the other) on a level of at least 256 small items of the frame, where the
// workgroup's ticket, group load and closing barrier are paid once per two items per wave (a
// level that crowded is far from the dependency chains' tail; round 5: 16 per group, or 8 on
// every level, measured slower, profiles/r05_ab_flow_groups.txt)
static uint32_t flow_small_group(const Level& lv)
{
    return lv.fcnt[2] - lv.tiny >= 256u ? 8u : 4u;
}
// k_flow groups of a level: its large items one each, its tiny items FLOW_TINY_G a group (four
// per wave, 16 lanes each), its other small items flow_small_group() a group
static size_t flow_groups(const Level& lv)
{
    const uint32_t G = flow_small_group(lv), rest = lv.fcnt[2] - lv.tiny;
    return lv.fcnt[1] + (lv.tiny + FLOW_TINY_G - 1) / FLOW_TINY_G + (rest + G - 1) / G;
}

// AV1R_SCHED_CHECK=1 (debug aid): the invariants k_flow relies on, checked on the host for a
// frame's flow schedule -- every index in range, every dependency (listed or through an edge
// granule) in an earlier k_flow group, residual tiles inside the residual buffer.  Prints
// the violations found and a summary line.
static void schedule_check(av1r_ctx* c, const av1r_frame_batch* b)
{
    long bad = 0;
    auto report = [&](const char* what, size_t i, long a, long b2) {
        if (bad++ < 20) fprintf(stderr, "av1r sched check: %s (item %zu: %ld %ld)\n", what, i, a, b2);
    };
    const size_t ni = c->items.size();
    std::vector<int64_t> grp(ni, -1);
    int64_t g = 0;
    for (size_t l = 0; l < c->levels.size(); l++) {
        const Level& lv = c->levels[l];
        if (lv.off[0] + lv.cnt[0] > c->tiles.size()) report("tiles range", l, lv.off[0], lv.cnt[0]);
        if (lv.off[1] + lv.cnt[1] > ni || lv.off[2] != lv.off[1] + lv.cnt[1] || lv.off[2] + lv.cnt[2] > ni)
            report("items range", l, lv.off[1], lv.cnt[1]);
        if (lv.fcnt[1] > lv.cnt[1] || lv.fcnt[2] > lv.cnt[2]) report("flow counts", l, lv.fcnt[1], lv.fcnt[2]);
        for (uint32_t q = 0; q < lv.fcnt[1]; q++) grp[lv.off[1] + q] = g++;
        if (lv.tiny > lv.fcnt[2]) report("tiny count", l, lv.tiny, lv.fcnt[2]);
        for (uint32_t q = 0; q < lv.tiny; q++) {
            grp[lv.off[2] + q] = g + q / FLOW_TINY_G;
            if (!(c->items[lv.off[2] + q].hflags & AV1R_WI_TINY)) report("tiny item", lv.off[2] + q, l, q);
        }
        g += (lv.tiny + FLOW_TINY_G - 1) / FLOW_TINY_G;
        const uint32_t G = flow_small_group(lv);
        for (uint32_t q = lv.tiny; q < lv.fcnt[2]; q++) grp[lv.off[2] + q] = g + (q - lv.tiny) / G;
        g += (lv.fcnt[2] - lv.tiny + G - 1) / G;
    }
    for (uint32_t t : c->tiles)
        if (AV1R_ITEM_KIND(t) != AV1R_ITEM_INTER || (AV1R_ITEM_INDEX(t) >> 4) >= b->n_blocks) report("tile code", 0, t, b->n_blocks);
    for (size_t i = 0; i < ni; i++) {
        const WorkItem& w = c->items[i];
        const uint32_t kind = AV1R_ITEM_KIND(w.code), idx = AV1R_ITEM_INDEX(w.code);
        if (kind == AV1R_ITEM_TB ? idx >= b->n_tbs : kind == AV1R_ITEM_II ? idx >= b->n_blocks : true) report("item code", i, w.code, 0);
        if (w.block >= b->n_blocks) report("item block", i, w.block, b->n_blocks);
        if (grp[i] < 0) continue;  // (not a k_flow item)
        if ((size_t)w.dep_off + w.dep_cnt > c->deps.size()) report("deps range", i, w.dep_off, w.dep_cnt);
        for (uint32_t d = 0; d < w.dep_cnt && (size_t)w.dep_off + d < c->deps.size(); d++) {
            const uint32_t p = c->deps[w.dep_off + d];
            if (p >= i || grp[p] < 0 || grp[p] >= grp[i]) report("listed dependency order", i, p, p < ni ? grp[p] : -1);
        }
        if (c->granOk && kind == AV1R_ITEM_TB) {
            const uint32_t ro = w.dep_off >= 1 ? c->deps[w.dep_off - 1] : 0;
            const size_t area = (size_t)av1r_tx_w[w.tx_size] * av1r_tx_h[w.tx_size];
            if (ro != ~0u && (size_t)ro + area > c->resElems) report("residual tile", i, ro, (long)c->resElems);
            if ((ro == ~0u) != (w.coef_cnt == 0)) report("residual presence", i, ro, w.coef_cnt);
        }
        const int32_t node = kind == AV1R_ITEM_TB ? c->nodeOfTb[idx] : kind == AV1R_ITEM_II ? c->nodeOfBlk[idx] : -1;
        if (node < 0 || c->edgeStart.size() <= (size_t)node + 1) continue;
        for (uint32_t e = c->edgeStart[node]; e < c->edgeStart[node + 1]; e++) {
            const int32_t pn = c->edgeDeps[e];
            const int32_t p = pn >= 0 && (size_t)pn < c->nodePos.size() ? c->nodePos[pn] : -1;
            if (p < 0 || grp[p] < 0 || grp[p] >= grp[i]) report("edge producer order", i, p, p >= 0 ? grp[p] : -1);
        }
    }
    fprintf(stderr, "av1r sched check: %zu items, %zu tiles, %lld groups, %ld violations\n", ni, c->tiles.size(), (long long)g, bad);
    static const bool chains = getenv("AV1R_SCHED_CHECK") && atoi(getenv("AV1R_SCHED_CHECK")) >= 2;
    if (chains) {
        // (debug aid) the longest dependency chain in items, and with the hops between items of
        // one block free (as if a block's items ran in one wave, one after the other)
        std::vector<int32_t> depth(ni, 1), depthB(ni, 1);
        int32_t maxD = 0, maxB = 0;
        for (size_t i = 0; i < ni; i++) {
            const WorkItem& w = c->items[i];
            const uint32_t kind = AV1R_ITEM_KIND(w.code), idx = AV1R_ITEM_INDEX(w.code);
            const int32_t node = kind == AV1R_ITEM_TB ? c->nodeOfTb[idx] : kind == AV1R_ITEM_II ? c->nodeOfBlk[idx] : -1;
            auto dep = [&](int32_t p) {
                if (p < 0 || (size_t)p >= i) return;
                depth[i] = std::max(depth[i], depth[p] + 1);
                depthB[i] = std::max(depthB[i], depthB[p] + (c->items[p].block == w.block ? 0 : 1));
            };
            for (uint32_t d = 0; d < w.dep_cnt; d++) dep((int32_t)c->deps[w.dep_off + d]);
            if (node >= 0 && c->edgeStart.size() > (size_t)node + 1)
                for (uint32_t e = c->edgeStart[node]; e < c->edgeStart[node + 1]; e++) {
                    const int32_t pn = c->edgeDeps[e];
                    dep(pn >= 0 && (size_t)pn < c->nodePos.size() ? c->nodePos[pn] : -1);
                }
            maxD = std::max(maxD, depth[i]);
            maxB = std::max(maxB, depthB[i]);
        }
        fprintf(stderr, "av1r sched chains: %zu levels, longest chain %d items, %d with a block's own hops free\n", c->levels.size(), maxD,
            maxB);
        // time model of the critical path (us): an item 6 (records, wait, gather, predict,
        // store, hand-off); a block-plane chain of small TBs run by one wave: 6 for its first
        // TB and 1.7 for each next one, the chain starting once every external producer of any
        // of its TBs is done
        std::vector<double> fin(ni, 0.0);
        std::vector<int32_t> chainOf(ni, -1);
        double tItems = 0, tChains = 0;
        {
            std::vector<double> f1(ni, 0.0);
            for (size_t i = 0; i < ni; i++) {
                const WorkItem& w = c->items[i];
                double st = 0;
                auto ext = [&](int32_t p) { if (p >= 0 && (size_t)p < i) st = std::max(st, f1[p]); };
                for (uint32_t d = 0; d < w.dep_cnt; d++) ext((int32_t)c->deps[w.dep_off + d]);
                const uint32_t kind = AV1R_ITEM_KIND(w.code), idx = AV1R_ITEM_INDEX(w.code);
                const int32_t node = kind == AV1R_ITEM_TB ? c->nodeOfTb[idx] : kind == AV1R_ITEM_II ? c->nodeOfBlk[idx] : -1;
                if (node >= 0)
                    for (uint32_t e = c->edgeStart[node]; e < c->edgeStart[node + 1]; e++)
                        ext(c->edgeDeps[e] >= 0 && (size_t)c->edgeDeps[e] < c->nodePos.size() ? c->nodePos[c->edgeDeps[e]] : -1);
                f1[i] = st + 6.0;
                tItems = std::max(tItems, f1[i]);
            }
            // chains: items in decode order (TB index order) of one block and plane, small TBs
            std::vector<int32_t> byTb(b->n_tbs, -1);
            for (size_t i = 0; i < ni; i++)
                if (AV1R_ITEM_KIND(c->items[i].code) == AV1R_ITEM_TB) byTb[AV1R_ITEM_INDEX(c->items[i].code)] = (int32_t)i;
            std::vector<std::vector<int32_t>> chainItems;
            for (uint32_t ti = 0; ti < b->n_tbs; ti++) {
                const int32_t i = byTb[ti];
                if (i < 0) continue;
                const WorkItem& w = c->items[i];
                const bool small = av1r_tx_w[w.tx_size] <= 16 && av1r_tx_h[w.tx_size] <= 16;
                const int32_t prevI = ti ? byTb[ti - 1] : -1;
                const bool cont = small && prevI >= 0 && c->items[prevI].block == w.block && c->items[prevI].plane == w.plane &&
                                  chainOf[prevI] >= 0 && chainItems[chainOf[prevI]].size() < 63;
                if (cont) {
                    chainOf[i] = chainOf[prevI];
                    chainItems[chainOf[i]].push_back(i);
                } else if (small) {
                    chainOf[i] = (int32_t)chainItems.size();
                    chainItems.push_back({i});
                }
            }
            // finish times in decode (node) order, which every dependency follows; a chain's
            // start waits for its externals (all its TBs')
            std::vector<double> chainStart(chainItems.size(), -1.0);
            for (size_t nd = 0; nd < c->nodePos.size(); nd++) {
                if (c->nodePos[nd] < 0) continue;
                const size_t i = (size_t)c->nodePos[nd];
                const WorkItem& w = c->items[i];
                auto externals = [&](size_t it, double& st) {
                    const WorkItem& x = c->items[it];
                    auto ext = [&](int32_t p) {
                        if (p < 0 || (size_t)p >= ni) return;
                        if (chainOf[it] >= 0 && chainOf[p] == chainOf[it]) return;  // internal
                        st = std::max(st, fin[p]);
                    };
                    for (uint32_t d = 0; d < x.dep_cnt; d++) ext((int32_t)c->deps[x.dep_off + d]);
                    const uint32_t kind = AV1R_ITEM_KIND(x.code), idx = AV1R_ITEM_INDEX(x.code);
                    const int32_t node = kind == AV1R_ITEM_TB ? c->nodeOfTb[idx] : kind == AV1R_ITEM_II ? c->nodeOfBlk[idx] : -1;
                    if (node >= 0)
                        for (uint32_t e = c->edgeStart[node]; e < c->edgeStart[node + 1]; e++)
                            ext(c->edgeDeps[e] >= 0 && (size_t)c->edgeDeps[e] < c->nodePos.size() ? c->nodePos[c->edgeDeps[e]] : -1);
                };
                const int32_t ch = chainOf[i];
                if (ch < 0) {
                    double st = 0;
                    externals(i, st);
                    fin[i] = st + 6.0;
                } else {
                    const auto& v = chainItems[ch];
                    if (chainStart[ch] < 0) {
                        double st = 0;
                        for (int32_t it : v) externals((size_t)it, st);  // (externals precede the chain in item order)
                        chainStart[ch] = st;
                    }
                    size_t k = 0;
                    while (v[k] != (int32_t)i) k++;
                    fin[i] = chainStart[ch] + 6.0 + 1.7 * (double)k;
                }
                (void)w;
                tChains = std::max(tChains, fin[i]);
            }
        }
        fprintf(stderr, "av1r sched chains: critical path (time model) items %.0f us, block-plane chains %.0f us\n", tItems, tChains);
    }
}

// the context's frames run on k_flow (av1r_set_schedule; default: k_flow, AV1R_FLOW=0 the
// level launches)
static bool flow_schedule(const av1r_ctx* c)
{
    static const bool flowEnv = !getenv("AV1R_FLOW") || atoi(getenv("AV1R_FLOW")) != 0;
    return c->schedule >= 0 ? c->schedule == 1 : flowEnv;
}

static void build_schedule(av1r_ctx* c, const av1r_frame_batch* b, bool allowGran = true, bool flowOnly = false)
{
    const av1r_frame_hdr* h = b->hdr;
    PackClock clk;
    if (flowOnly)
        for (uint32_t i = 0; i < b->n_blocks && flowOnly; i++) flowOnly = !(b->blocks[i].flags & AV1R_BLK_INTRABC);
    c->levelsOk = !flowOnly;
    for (int p = 0; p < 3; p++) {
        int sub = p ? 1 : 0;
        c->mapW[p] = (((h->mi_stride * 4) >> sub) + 64) / 4;
        c->mapH[p] = (((h->mi_rows_alloc * 4) >> sub) + 64) / 4;
        // k_flow only (flowOnly): the levels just order the items, dependencies carry the
        // hand-offs, so the inter predictions' level 0 is the map's initial value and the
        // plain inter blocks need not be painted (below)
        c->umap[p].assign((size_t)c->mapW[p] * c->mapH[p], av1r_ctx::MapUnit{-1, (int16_t)(flowOnly ? 0 : -1), 0, 0});
    }
    c->granOk = allowGran;
    c->nodeMask.clear();
    uint32_t nm[12] = {};  // mask words of the node being built
    c->nodeDepStart.assign(1, 0);
    c->nodeDeps.clear();
    c->nodeLvl.clear();
    c->edgeDeps.clear();
    c->edgeStart.assign(1, 0);
    // critical-path order (below): each item moves half of its slack toward its latest level
    // (round 5: 0 / 50 / 100 % measured the same device time, 50 the best host-inclusive rate)
    const int alapPct = 50;
    const bool alap = flowOnly;
    c->nodeOfTb.assign(b->n_tbs, -1);
    c->nodeOfBlk.assign(b->n_blocks, -1);
    std::vector<int32_t> dl;  // dependencies of the node being built
    auto owners = [&](int p, int x0, int y0, int x1, int y1) {  // inclusive 4x4-unit rect
        x0 = std::max(x0, 0);
        y0 = std::max(y0, 0);
        x1 = std::min(x1, c->mapW[p] - 1);
        y1 = std::min(y1, c->mapH[p] - 1);
        for (int y = y0; y <= y1; y++) {
            const av1r_ctx::MapUnit* row = &c->umap[p][(size_t)y * c->mapW[p]];
            int32_t last = -1;
            for (int x = x0; x <= x1; x++)
                if (row[x].owner >= 0 && row[x].owner != last) dl.push_back(last = row[x].owner);
        }
    };
    // the owners of the pixels an intra prediction reads (coop_intra_edges): with granules,
    // mask words nm[4 * slot ..] instead of dependencies (coop_intra_edges_gran's runs)
    auto edge_owners = [&](int p, int x, int y, int w, int h, bool hL, bool hA, bool hAR, bool hBL, int slot, int need) {
        if (!c->granOk) {
            if (hA && (need & 1)) owners(p, x >> 2, (y - 1) >> 2, (x + (hAR ? 2 * w : w) - 1) >> 2, (y - 1) >> 2);
            if (hL && (need & 2)) owners(p, (x - 1) >> 2, y >> 2, (x - 1) >> 2, (y + (hBL ? 2 * h : h) - 1) >> 2);
            if (hA && hL && (need & 4)) owners(p, (x - 1) >> 2, (y - 1) >> 2, (x - 1) >> 2, (y - 1) >> 2);
            return;
        }
        uint32_t* m = nm + 4 * slot;
        auto run = [&](int u0, int u1, bool horiz, uint32_t* mw) {  // units u0..u1 of row / column
            if (u1 - u0 >= 32) c->granOk = false;
            for (int u = u0; u <= u1 && u - u0 < 32; u++) {
                const int ux = horiz ? u : (x - 1) >> 2, uy = horiz ? (y - 1) >> 2 : u;
                if (ux < 0 || uy < 0 || ux >= c->mapW[p] || uy >= c->mapH[p]) continue;
                const size_t i = (size_t)uy * c->mapW[p] + ux;
                const av1r_ctx::MapUnit& mu = c->umap[p][i];
                if (mu.owner < 0) continue;
                *mw |= 1u << (u - u0);
                if (alap) c->edgeDeps.push_back(mu.owner);
                if (!(mu.emit & (horiz ? 1 : 2))) c->granOk = false;
            }
        };
        // above run: row (y-1)/4 from x/4; left run: column (x-1)/4 from y/4; the corner
        // pixel (x-1, y-1) separately (m[1]: bit 0 written in the launch, bit 1 its
        // granule is its owner's right column instead of its bottom row)
        if (hA && (need & 1)) run(x >> 2, (x + (hAR ? 2 * w : w) - 1) >> 2, true, m);
        if (hL && (need & 2)) run(y >> 2, (y + (hBL ? 2 * h : h) - 1) >> 2, false, m + 2);
        if (hA && hL && (need & 4)) {
            const size_t i = (size_t)((y - 1) >> 2) * c->mapW[p] + ((x - 1) >> 2);
            const av1r_ctx::MapUnit& mu = c->umap[p][i];
            if (mu.owner >= 0) {
                m[1] = (mu.emit & 1) ? 1u : 3u;
                if (!mu.emit) c->granOk = false;
                if (alap) c->edgeDeps.push_back(mu.owner);
            }
        }
    };
    auto own_set = [&](int p, int x0, int y0, int w4, int h4, int32_t node) {
        if (x0 + w4 > c->mapW[p] || y0 + h4 > c->mapH[p]) c->granOk = false;  // its granules would not fit
        int x1 = std::min(x0 + w4, c->mapW[p]), y1 = std::min(y0 + h4, c->mapH[p]);
        for (int y = y0; y < y1; y++) {
            av1r_ctx::MapUnit* row = &c->umap[p][(size_t)y * c->mapW[p]];
            const uint8_t last = y == y0 + h4 - 1 ? 1 : 0;
            for (int x = x0; x < x1; x++) {
                row[x].owner = node;
                row[x].emit = last | (x == x0 + w4 - 1 ? 2 : 0);
            }
        }
    };
    auto end_node = [&]() {  // closes the node's dependency list; returns its id
        if (dl.size() > 1) {
            std::sort(dl.begin(), dl.end());
            dl.erase(std::unique(dl.begin(), dl.end()), dl.end());
        }
        if (!dl.empty()) c->nodeDeps.insert(c->nodeDeps.end(), dl.begin(), dl.end());
        dl.clear();
        const size_t nmo = c->nodeMask.size();
        c->nodeMask.resize(nmo + 12);
        memcpy(c->nodeMask.data() + nmo, nm, sizeof(nm));
        memset(nm, 0, sizeof(nm));
        c->nodeDepStart.push_back((uint32_t)c->nodeDeps.size());
        c->edgeStart.push_back((uint32_t)c->edgeDeps.size());
        return (int32_t)c->nodeDepStart.size() - 2;
    };
    for (auto* v : {&c->lvP, &c->lvB, &c->lvT})
        for (auto& l : *v) l.clear();
    auto region_max = [&](int p, int x0, int y0, int x1, int y1) {  // inclusive 4x4-unit rect
        x0 = std::max(x0, 0);
        y0 = std::max(y0, 0);
        x1 = std::min(x1, c->mapW[p] - 1);
        y1 = std::min(y1, c->mapH[p] - 1);
        int m = -1;
        for (int y = y0; y <= y1; y++) {
            const av1r_ctx::MapUnit* row = &c->umap[p][(size_t)y * c->mapW[p]];
            for (int x = x0; x <= x1; x++) m = std::max<int>(m, row[x].lvl);
        }
        return m;
    };
    auto region_set = [&](int p, int x0, int y0, int w4, int h4, int lv) {
        int x1 = std::min(x0 + w4, c->mapW[p]), y1 = std::min(y0 + h4, c->mapH[p]);
        for (int y = y0; y < y1; y++) {
            av1r_ctx::MapUnit* row = &c->umap[p][(size_t)y * c->mapW[p]];
            for (int x = x0; x < x1; x++) row[x].lvl = (int16_t)lv;
        }
    };
    auto region_own_set = [&](int p, int x0, int y0, int w4, int h4, int lv, int32_t node) {  // both at once
        if (x0 + w4 > c->mapW[p] || y0 + h4 > c->mapH[p]) c->granOk = false;
        int x1 = std::min(x0 + w4, c->mapW[p]), y1 = std::min(y0 + h4, c->mapH[p]);
        for (int y = y0; y < y1; y++) {
            av1r_ctx::MapUnit* row = &c->umap[p][(size_t)y * c->mapW[p]];
            const uint8_t last = y == y0 + h4 - 1 ? 1 : 0;
            for (int x = x0; x < x1; x++) row[x] = av1r_ctx::MapUnit{node, (int16_t)lv, (uint8_t)(last | (x == x0 + w4 - 1 ? 2 : 0)), 0};
        }
    };
    // Latest level among the pixels coop_intra_predict reads for a w x h prediction at
    // pixel (x, y) of plane p with the given edge availability (IntraPredict.cpp:563-631):
    // row y-1 over [x-1 | x, x + (AR ? 2w : w) - 1], column x-1 over [y-1 | y, y + (BL ? 2h : h) - 1];
    // with only one edge available its neighbouring corner pixel stands in for the other.
    auto edge_level = [&](int p, int x, int y, int w, int h, bool hL, bool hA, bool hAR, bool hBL, int need) {
        int m = -1;
        if (hA && (need & 1)) m = std::max(m, region_max(p, x >> 2, (y - 1) >> 2, (x + (hAR ? 2 * w : w) - 1) >> 2, (y - 1) >> 2));
        if (hL && (need & 2)) m = std::max(m, region_max(p, (x - 1) >> 2, y >> 2, (x - 1) >> 2, (y + (hBL ? 2 * h : h) - 1) >> 2));
        if (hA && hL && (need & 4)) m = std::max(m, region_max(p, (x - 1) >> 2, (y - 1) >> 2, (x - 1) >> 2, (y - 1) >> 2));
        return m;
    };
    // granule mode: edge_level and edge_owners in one walk over the same units (the above
    // run, the left run, the corner); returns the latest level
    auto edge_scan = [&](int p, int x, int y, int w, int h, bool hL, bool hA, bool hAR, bool hBL, int slot, int need) {
        int m = -1;
        uint32_t* mw = nm + 4 * slot;
        const int W = c->mapW[p], H = c->mapH[p];
        const av1r_ctx::MapUnit* map = c->umap[p].data();
        auto unit = [&](int ux, int uy, int bit, uint32_t* word, uint8_t need) {
            if (ux < 0 || uy < 0 || ux >= W || uy >= H) return;
            const av1r_ctx::MapUnit& mu = map[(size_t)uy * W + ux];
            m = std::max<int>(m, mu.lvl);
            if (mu.owner < 0) return;
            *word |= 1u << bit;
            if (!(mu.emit & need)) c->granOk = false;
            if (alap) c->edgeDeps.push_back(mu.owner);
        };
        if (hA && (need & 1)) {
            const int u0 = x >> 2, u1 = (x + (hAR ? 2 * w : w) - 1) >> 2, uy = (y - 1) >> 2;
            if (u1 - u0 >= 32) c->granOk = false;
            for (int u = u0; u <= u1 && u - u0 < 32; u++) unit(u, uy, u - u0, mw, 1);
        }
        if (hL && (need & 2)) {
            const int u0 = y >> 2, u1 = (y + (hBL ? 2 * h : h) - 1) >> 2, ux = (x - 1) >> 2;
            if (u1 - u0 >= 32) c->granOk = false;
            for (int u = u0; u <= u1 && u - u0 < 32; u++) unit(ux, u, u - u0, mw + 2, 2);
        }
        if (hA && hL && (need & 4)) {
            const int ux = (x - 1) >> 2, uy = (y - 1) >> 2;
            if (ux >= 0 && uy >= 0 && ux < W && uy < H) {
                const av1r_ctx::MapUnit& mu = map[(size_t)uy * W + ux];
                m = std::max<int>(m, mu.lvl);
                if (mu.owner >= 0) {
                    mw[1] = (mu.emit & 1) ? 1u : 3u;
                    if (!mu.emit) c->granOk = false;
                    if (alap) c->edgeDeps.push_back(mu.owner);
                }
            }
        }
        return m;
    };
    auto push = [&](std::vector<std::vector<uint32_t>>& v, int lv, uint32_t item) {
        if ((int)v.size() <= lv) v.resize(lv + 1);
        v[lv].push_back(item);
    };
    int globalMax = -1;
    clk.lap(PP_SCHED_INIT);
    for (uint32_t bi = 0; bi < b->n_blocks; bi++) {
        const av1r_block& blk = b->blocks[bi];
        const bool inter = blk.flags & AV1R_BLK_INTER;
        const int nPlanes = (blk.flags & AV1R_BLK_HAS_CHROMA) ? 3 : 1;
        int blkLevel = -1;  // level after which the block's prediction is complete
        if (inter) {
            const bool isII = blk.ref_frame[1] == AV1R_INTRA_FRAME;
            // intra block copy reads already-decoded pixels of the current frame
            const int pLevel = (blk.flags & AV1R_BLK_INTRABC) ? globalMax + 1 : 0;
            const int bw = av1r_num4x4w[blk.mi_size] * 4, bh = av1r_num4x4h[blk.mi_size] * 4;
            for (int ty = 0; ty < (bh + 31) / 32; ty++)
                for (int tx = 0; tx < (bw + 31) / 32; tx++)
                    push(c->lvP, pLevel, AV1R_ITEM(AV1R_ITEM_INTER, (bi << 4) | (ty << 2) | tx));
            blkLevel = pLevel;
            int32_t iiNode = -1;
            if (isII) {
                int dep = pLevel;
                for (int p = 0; p < nPlanes; p++) {
                    int sub = p ? 1 : 0;
                    int psz = p ? av1r_ss420[blk.mi_size] : blk.mi_size;
                    bool hL = p ? (blk.flags & AV1R_BLK_AVAIL_L_UV) : (blk.flags & AV1R_BLK_AVAIL_L);
                    bool hA = p ? (blk.flags & AV1R_BLK_AVAIL_U_UV) : (blk.flags & AV1R_BLK_AVAIL_U);
                    const int ex = (blk.mi_col >> sub) * 4, ey = (blk.mi_row >> sub) * 4;
                    const int ew = av1r_num4x4w[psz] * 4, eh = av1r_num4x4h[psz] * 4;
                    // (the inter-intra modes read neither the above-right nor the below-left
                    // run, nor the corner: II_DC / V / H / SMOOTH)
                    const bool hAR = false, hBL = false;
                    const int need = 3;
                    dep = std::max(dep, edge_level(p, ex, ey, ew, eh, hL, hA, hAR, hBL, need));
                    edge_owners(p, ex, ey, ew, eh, hL, hA, hAR, hBL, p, need);
                }
                blkLevel = dep + 1;
                push(c->lvB, blkLevel, AV1R_ITEM(AV1R_ITEM_II, bi));
                iiNode = c->nodeOfBlk[bi] = end_node();
                c->nodeLvl.push_back(blkLevel);
            }
            globalMax = std::max(globalMax, blkLevel);
            // (flowOnly: a plain inter block is level 0 and owns nothing -- the maps' initial
            // values -- so it is not painted; blocks never overlap)
            if (!flowOnly || isII)
                for (int p = 0; p < nPlanes; p++) {
                    int sub = p ? 1 : 0;
                    int psz = p ? av1r_ss420[blk.mi_size] : blk.mi_size;
                    region_set(p, blk.mi_col >> sub, blk.mi_row >> sub, av1r_num4x4w[psz], av1r_num4x4h[psz], blkLevel);
                    own_set(p, blk.mi_col >> sub, blk.mi_row >> sub, av1r_num4x4w[psz], av1r_num4x4h[psz], iiNode);
                }
        }
        // (flowOnly: an inter block's transform blocks get no node, item or level -- k_resid
        // adds their residuals before k_flow)
        if (inter && flowOnly) continue;
        int lumaMax = -1;  // CFL reads this block's reconstructed luma
        for (uint32_t ti = blk.first_tb; ti < blk.first_tb + blk.n_tbs; ti++) {
            const av1r_tb& t = b->tbs[ti];
            const int p = t.plane;
            const int w = av1r_tx_w[t.tx_size], hh = av1r_tx_h[t.tx_size];
            int lv;
            if (inter) {
                if (!t.coef_cnt || flowOnly) continue;  // prediction only: nothing to add
                lv = blkLevel + 1;
                // the prediction it adds to: the inter tile (preceding launch) or the blend
                if (c->nodeOfBlk[bi] >= 0) dl.push_back(c->nodeOfBlk[bi]);
            } else {
                const bool pal = p ? blk.palette_size_uv : blk.palette_size_y;
                int dep = -1;
                if (!pal) {
                    const bool hL = t.flags & AV1R_TB_HAVE_LEFT, hA = t.flags & AV1R_TB_HAVE_ABOVE;
                    const int ang = intra_angle(blk, p);
                    const bool hAR = (t.flags & AV1R_TB_HAVE_AR) && ang > 0 && ang < 90;
                    const bool hBL = (t.flags & AV1R_TB_HAVE_BL) && ang > 180;
                    const int need = intra_needs(blk, p, hA, hL);
                    if (c->granOk) {
                        dep = edge_scan(p, t.x, t.y, w, hh, hL, hA, hAR, hBL, 0, need);
                    } else {
                        dep = edge_level(p, t.x, t.y, w, hh, hL, hA, hAR, hBL, need);
                        edge_owners(p, t.x, t.y, w, hh, hL, hA, hAR, hBL, 0, need);
                    }
                    if (p && blk.uv_mode == AV1R_UV_CFL_PRED) {  // the co-located luma (incl. sub-8x8 neighbours)
                        const int lx0 = t.x >> 1, ly0 = t.y >> 1, lx1 = (2 * (t.x + w) - 1) >> 2, ly1 = (2 * (t.y + hh) - 1) >> 2;
                        dep = std::max({dep, lumaMax, region_max(0, lx0, ly0, lx1, ly1)});
                        owners(0, lx0, ly0, lx1, ly1);
                        // (lumaMax: this block's luma TBs, all earlier nodes of the block)
                        for (uint32_t tj = blk.first_tb; tj < ti; tj++)
                            if (b->tbs[tj].plane == 0 && c->nodeOfTb[tj] >= 0) dl.push_back(c->nodeOfTb[tj]);
                    }
                }
                lv = dep + 1;
            }
            if (p == 0) lumaMax = std::max(lumaMax, lv);
            push(c->lvT, lv, AV1R_ITEM(AV1R_ITEM_TB, ti));
            globalMax = std::max(globalMax, lv);
            const int32_t node = c->nodeOfTb[ti] = end_node();
            c->nodeLvl.push_back(lv);
            // an inter TB's pixels are final before k_flow (k_inter + k_resid) unless the
            // block is inter-intra, whose blend item adds the residuals
            if (!inter) {
                region_own_set(p, t.x >> 2, t.y >> 2, w >> 2, hh >> 2, lv, node);
            } else {
                region_set(p, t.x >> 2, t.y >> 2, w >> 2, hh >> 2, lv);
                if (!inter) own_set(p, t.x >> 2, t.y >> 2, w >> 2, hh >> 2, node);
            }
        }
    }
    if (c->granOk != allowGran) {  // a unit without its granule: dependency flags throughout
        build_schedule(c, b, false, flowOnly);
        return;
    }
    // Critical-path order (flow-only frames).  k_flow hands its groups out
    // in level order, so an item of a long chain waits in the queue behind every item of the
    // levels before it, and the chain's tail runs alone after the bulk (a batched inter step:
    // levels 10-46 all released ~185 us into a 256 us launch, then one hop after another).
    // Each item moves toward the LATEST level it can have without lengthening the schedule,
    // L - height (height = the longest chain of consumers below it, through nodeDeps and the
    // edge producers recorded above; L = max(level + height)): to level + a * slack, slack =
    // L - height - level, a = alapPct / 100.  For a producer P of C, level(C) >= level(P) + 1
    // and L - height(C) >= L - height(P) + 1, so every such mix keeps C after P: the order stays
    // topological (k_flow's progress argument holds).  The items on the chains keep their level
    // (no slack) while those nothing waits for (height 0) move back, behind the chains' heads.
    if (alap && !c->nodeLvl.empty()) {
        const size_t nn = c->nodeLvl.size();
        c->nodeHeight.assign(nn, 0);
        int32_t* ht = c->nodeHeight.data();
        for (size_t n = nn; n-- > 0;) {  // decode order is topological: consumers after producers
            const int32_t hn = ht[n] + 1;
            for (uint32_t d = c->nodeDepStart[n]; d < c->nodeDepStart[n + 1]; d++) ht[c->nodeDeps[d]] = std::max(ht[c->nodeDeps[d]], hn);
            for (uint32_t d = c->edgeStart[n]; d < c->edgeStart[n + 1]; d++) ht[c->edgeDeps[d]] = std::max(ht[c->edgeDeps[d]], hn);
        }
        int L = 0;
        for (size_t n = 0; n < nn; n++) L = std::max(L, c->nodeLvl[n] + ht[n]);
        for (size_t n = 0; n < nn; n++) ht[n] = c->nodeLvl[n] + (L - ht[n] - c->nodeLvl[n]) * alapPct / 100;  // (the new level)
        auto relevel = [&](std::vector<std::vector<uint32_t>>& v, bool ii) {
            std::vector<std::vector<uint32_t>> out(std::max<size_t>(v.size(), (size_t)L + 1));
            for (auto& lvList : v)
                for (uint32_t code : lvList) {
                    const uint32_t idx = AV1R_ITEM_INDEX(code);
                    const int32_t node = ii ? c->nodeOfBlk[idx] : c->nodeOfTb[idx];
                    out[node >= 0 ? ht[node] : 0].push_back(code);
                }
            v.swap(out);
        };
        relevel(c->lvB, true);
        relevel(c->lvT, false);
        globalMax = std::max(globalMax, L);
    }
    const size_t nl = (size_t)(globalMax + 1);
    clk.lap(PP_SCHED_BLOCKS);
    for (auto* v : {&c->lvP, &c->lvB, &c->lvT})
        if (v->size() < nl) v->resize(nl);
    c->items.clear();
    c->tiles.clear();
    c->levels.assign(nl, Level());
    size_t nItems = 0, nTiles = 0;
    for (size_t l = 0; l < nl; l++) nItems += c->lvB[l].size() + c->lvT[l].size(), nTiles += c->lvP[l].size();
    c->items.reserve(nItems);
    c->tiles.reserve(nTiles);
    // stable partition of a level's list by a small class key (counting sort, one pass)
    std::vector<uint32_t> bk[5];
    auto partition = [&](std::vector<uint32_t>& v, int nk, uint32_t* counts, auto key) {
        for (int q = 0; q < nk; q++) bk[q].clear();
        for (uint32_t x : v) bk[key(x)].push_back(x);
        size_t o = 0;
        for (int q = 0; q < nk; q++) {
            counts[q] = (uint32_t)bk[q].size();
            std::copy(bk[q].begin(), bk[q].end(), v.begin() + o);
            o += bk[q].size();
        }
    };
    // inter tiles: [the rest][medium plain][small plain].  Plain = simple motion, no mask
    // compound, no intra block copy, no global warp: what k_inter_m / k_inter_s predict
    // (their frames' references must also be unscaled, checked per launch); small = both
    // luma sides <= 8, medium = both <= 16
    auto plainClass = [&](uint32_t code) {  // 0 k_inter, 1 medium, 2 small
        const av1r_block& blk = b->blocks[AV1R_ITEM_INDEX(code) >> 4];
        const int bs = blk.mi_size;
        if (av1r_num4x4w[bs] > 4 || av1r_num4x4h[bs] > 4) return 0;
        if (blk.motion_mode != AV1R_SIMPLE_TRANSLATION || (blk.flags & AV1R_BLK_INTRABC)) return 0;
        const av1r_block& info = blk;  // (its mode info)
        if (info.ref_frame[1] > AV1R_INTRA_FRAME && blk.compound_type != AV1R_COMPOUND_AVERAGE &&
            blk.compound_type != AV1R_COMPOUND_DISTANCE)
            return 0;
        if (blk.y_mode == AV1R_GLOBALMV || blk.y_mode == AV1R_GLOBAL_GLOBALMV)
            for (int r = 0; r < 2; r++)
                if (info.ref_frame[r] > AV1R_INTRA_FRAME && h->gm_type[info.ref_frame[r] & 7] > AV1R_GM_TRANSLATION)
                    return 0;
        return av1r_num4x4w[bs] <= 2 && av1r_num4x4h[bs] <= 2 ? 2 : 1;
    };
    // TB lists: [large intra][large inter][tiny][small intra][small inter]; large = a side >
    // 16; tiny (flow-only frames with granules, on a level of at least 256 small intra TBs):
    // an intra TB of at most 8x8 on k_flow's lean path -- not palette, not filter-intra
    // (intra_fast.h fi_ok) -- described by a TinyItem.  A tiny group's four items per wave run
    // in lock step, each row waiting for the others' edges: on the thin levels of a dependency
    // chain (a key frame: ~70 items per level) that lengthens every hop (measured: a 1080p key
    // frame 1.70 -> 3.09 ms with every level's tiny items in tiny groups), so they stay one per
    // wave there.
    bool tinyOk = false;
    auto smallIntra = [&](uint32_t code) {
        const av1r_tb& t = b->tbs[AV1R_ITEM_INDEX(code)];
        return av1r_tx_w[t.tx_size] <= 16 && av1r_tx_h[t.tx_size] <= 16 && !(b->blocks[t.block].flags & AV1R_BLK_INTER);
    };
    auto tbClass = [&](uint32_t code) {
        const av1r_tb& t = b->tbs[AV1R_ITEM_INDEX(code)];
        const av1r_block& blk = b->blocks[t.block];
        const bool inter = blk.flags & AV1R_BLK_INTER;
        if (av1r_tx_w[t.tx_size] > 16 || av1r_tx_h[t.tx_size] > 16) return inter ? 1 : 0;
        if (inter) return 4;
        const bool tiny = tinyOk && av1r_tx_w[t.tx_size] <= 8 && av1r_tx_h[t.tx_size] <= 8 &&
                          !(t.plane ? blk.palette_size_uv : blk.palette_size_y) && !(t.plane == 0 && (blk.flags & AV1R_BLK_FILTER_INTRA));
        return tiny ? 2 : 3;
    };
    for (size_t l = 0; l < nl; l++) {
        // order: inter tiles, then k_tb's large items, then its small ones
        uint32_t pc[4] = {}, tc[5] = {};
        partition(c->lvP[l], 3, pc, plainClass);
        c->levels[l].pl[0] = pc[1];
        c->levels[l].pl[1] = pc[2];
        std::vector<uint32_t>& T = c->lvT[l];
        tinyOk = false;
        if (flowOnly && c->granOk && T.size() >= 256) {
            size_t nsi = 0;
            for (uint32_t code : T) nsi += smallIntra(code);
            tinyOk = nsi >= 256;
        }
        partition(T, 5, tc, tbClass);
        const uint32_t nLargeT = tc[0] + tc[1], nLargeIntra = tc[0], nSmallIntra = tc[2] + tc[3];
        c->levels[l].tiny = tc[2];
        c->levels[l].off[0] = (uint32_t)c->tiles.size();
        c->levels[l].cnt[0] = (uint32_t)c->lvP[l].size();
        c->tiles.insert(c->tiles.end(), c->lvP[l].begin(), c->lvP[l].end());
        c->levels[l].off[1] = (uint32_t)c->items.size();
        c->levels[l].cnt[1] = (uint32_t)c->lvB[l].size() + nLargeT;
        c->levels[l].off[2] = c->levels[l].off[1] + c->levels[l].cnt[1];
        c->levels[l].cnt[2] = (uint32_t)T.size() - nLargeT;
        c->levels[l].fcnt[0] = 0;
        c->levels[l].fcnt[1] = (uint32_t)c->lvB[l].size() + nLargeIntra;
        c->levels[l].fcnt[2] = nSmallIntra;
        for (auto* v : {&c->lvB, &c->lvT}) {
            for (uint32_t code : (*v)[l]) {
                WorkItem w;
                memset(&w, 0, sizeof(w));
                w.code = code;
                const uint32_t idx = AV1R_ITEM_INDEX(code);
                switch (AV1R_ITEM_KIND(code)) {
                case AV1R_ITEM_II: w.block = idx; break;
                default: {
                    const av1r_tb& t = b->tbs[idx];
                    const av1r_block& blk = b->blocks[t.block];
                    w.block = t.block;
                    w.coef_off = t.coef_off;
                    w.x = t.x;
                    w.y = t.y;
                    w.coef_cnt = t.coef_cnt;
                    w.plane = t.plane;
                    w.tx_size = t.tx_size;
                    w.tx_type = t.tx_type;
                    w.flags = t.flags;
                    w.pred = (blk.flags & AV1R_BLK_INTER) ? AV1R_PRED_INTER
                           : (t.plane ? blk.palette_size_uv : blk.palette_size_y) ? AV1R_PRED_PALETTE
                                                                                  : AV1R_PRED_INTRA;
                }
                }
                c->items.push_back(w);
            }
        }
        for (uint32_t q = 0; q < tc[2]; q++) c->items[c->levels[l].off[2] + q].hflags = AV1R_WI_TINY;
    }
    c->nLevelsLast = (int)nl;
    clk.lap(PP_SCHED_ITEMS);
    // k_resid: residual tiles for intra TBs and the TBs of inter-intra blocks; the other
    // inter TBs are added in place
    c->tbRes.assign(b->n_tbs, ~0u);
    // (k_resid_s's list: the 4x4 TBs first, 64 per workgroup at 4 lanes each -- half the
    // TBs with coefficients --, then the 8x8 / 8x4 / 4x8 ones, 32 per workgroup at 8 lanes
    // (with 16, half the lanes idled through both passes of an 8x8), then the others up to
    // 16x16, 16 per workgroup at 16 lanes)
    c->residS.clear();
    c->residL.clear();
    c->residT.clear();
    c->residE.clear();
    c->residM.clear();
    c->resElems = 0;
    for (uint32_t ti = 0; ti < b->n_tbs; ti++) {
        const av1r_tb& t = b->tbs[ti];
        if (!t.coef_cnt) continue;
        const int w = av1r_tx_w[t.tx_size], hh = av1r_tx_h[t.tx_size];
        const bool inPlace = (b->blocks[t.block].flags & AV1R_BLK_INTER) && c->nodeOfBlk[t.block] < 0;
        if (!inPlace) {
            c->tbRes[ti] = (uint32_t)c->resElems;
            c->resElems += (size_t)w * hh;
        }
        (t.tx_size == AV1R_TX_4X4 ? c->residT : w <= 8 && hh <= 8 ? c->residE : w <= 16 && hh <= 16 ? c->residS
         : w <= 32 && hh <= 32 ? c->residM : c->residL).push_back(ti);
    }
    // (k_resid_l: two TBs of at most 32x32 per 64-lane workgroup, 32 lanes each -- one lane
    // per row / column, so a 32-wide TB left half of 64 idle --, then the 64-sided ones)
    while (c->residM.size() % 2) c->residM.push_back(~0u);
    c->nResidM = (uint32_t)(c->residM.size() / 2);
    c->residL.insert(c->residL.begin(), c->residM.begin(), c->residM.end());
    c->residL.insert(c->residL.begin(), c->nResidM);  // (its head: the pairs' workgroup count)
    while (c->residT.size() % 64) c->residT.push_back(~0u);
    while (c->residE.size() % 32) c->residE.push_back(~0u);
    while (c->residS.size() % 16) c->residS.push_back(~0u);
    c->nResidT = (uint32_t)(c->residT.size() / 64);
    c->nResidE = (uint32_t)(c->residE.size() / 32);
    c->residS.insert(c->residS.begin(), c->residE.begin(), c->residE.end());
    c->residS.insert(c->residS.begin(), c->residT.begin(), c->residT.end());
    // k_flow: dependency lists as item positions (every dependency is an earlier item: it
    // has a lower level); inter tiles after level 0 (intra block copy) keep the frame on
    // the level launches
    c->flowOk = c->resElems < 0xffffffffu;
    for (size_t l = 1; l < nl; l++) c->flowOk &= c->lvP[l].empty();
    c->nodePos.assign(c->nodeDepStart.size() - 1, -1);
    for (size_t i = 0; i < c->items.size(); i++) {
        const uint32_t code = c->items[i].code;
        const uint32_t idx = AV1R_ITEM_INDEX(code);
        const int32_t node = AV1R_ITEM_KIND(code) == AV1R_ITEM_TB ? c->nodeOfTb[idx]
                           : AV1R_ITEM_KIND(code) == AV1R_ITEM_II ? c->nodeOfBlk[idx] : -1;
        if (node >= 0) c->nodePos[node] = (int32_t)i;
    }
    c->deps.clear();
    for (size_t i = 0; i < c->items.size() && c->flowOk; i++) {
        WorkItem& w = c->items[i];
        const uint32_t code = w.code;
        const uint32_t idx = AV1R_ITEM_INDEX(code);
        const int32_t node = AV1R_ITEM_KIND(code) == AV1R_ITEM_TB ? c->nodeOfTb[idx]
                           : AV1R_ITEM_KIND(code) == AV1R_ITEM_II ? c->nodeOfBlk[idx] : -1;
        if (node < 0) continue;
        const uint32_t d0 = c->nodeDepStart[node], d1 = c->nodeDepStart[node + 1];
        if (d1 - d0 > 0xffff) {
            c->flowOk = false;
            break;
        }
        if (c->granOk) {  // the mask words precede the list: 12 for a blend, 4 for a TB
            const uint32_t* m = &c->nodeMask[(size_t)node * 12];
            c->deps.insert(c->deps.end(), m, m + (AV1R_ITEM_KIND(code) == AV1R_ITEM_II ? 12 : 4));
            // a TB's fourth word (no edge run uses it): its residual tile's offset, so that
            // k_flow fetches the residual with the masks' scalar load instead of through tb_res
            if (AV1R_ITEM_KIND(code) == AV1R_ITEM_TB) c->deps.back() = w.coef_cnt ? c->tbRes[idx] : ~0u;
        }
        w.dep_off = (uint32_t)c->deps.size();
        w.dep_cnt = (uint16_t)(d1 - d0);
        for (uint32_t d = d0; d < d1; d++) {
            const int32_t pos = c->nodePos[c->nodeDeps[d]];
            if (pos < 0 || pos >= (int32_t)i) {  // cannot happen: levels order the items
                c->flowOk = false;
                break;
            }
            c->deps.push_back((uint32_t)pos);
            c->items[pos].pub = 1;
        }
    }
    clk.lap(PP_SCHED_DEPS);
    if (flowOnly && !c->flowOk) {
        build_schedule(c, b, allowGran, false);  // k_flow cannot take it: levels too
        return;
    }
    static const bool check = getenv("AV1R_SCHED_CHECK") != nullptr;
    if (check && c->flowOk) schedule_check(c, b);
}

// ------------------------------------------------------------------------------------
// validate + schedule + pack into `host` (capacity checked by caller via size query)
static int pack_frame(av1r_ctx* c, const av1r_frame_batch* b, Prepared& P, uint8_t* host, uint8_t* dev, size_t* need)
{
    const av1r_frame_hdr* h = b->hdr;
    const size_t szHdr = align256(sizeof(av1r_frame_hdr));
    const size_t szMi = align256(sizeof(av1r_mi) * (size_t)h->mi_stride * h->mi_rows_alloc);
    // the deblocking edge codes (k_lfcode): a byte per (pass, plane, 4x4 unit), device-filled
    // the blocks in the device's record (DevBlock), the warp parameters and TB ranges of the
    // LOCAL_VALID / INTERINTRA blocks beside them (bext, 8 words each)
    const uint32_t extFlags = AV1R_BLK_LOCAL_VALID | AV1R_BLK_INTERINTRA;
    size_t nExt = 0;
    for (uint32_t i = 0; i < b->n_blocks; i++) nExt += (b->blocks[i].flags & extFlags) != 0;
    const size_t szBlk = align256(sizeof(DevBlock) * (size_t)b->n_blocks);
    const size_t szExt = align256(32 * nExt + 4);
    const size_t szTb = align256(sizeof(DevTb) * (size_t)b->n_tbs);
    if (!host) {
        // the coefficient widths: 16 bits when a level fits 6 signed bits, i.e. (level << 10
        // | pos) fits int16.  One vectorised OR over the whole array first; only a frame with
        // some wider level classifies its TBs
        const uint32_t* cf = b->coefs;
        if (!c->wideKnown || c->tbWide.size() != b->n_tbs) {  // (validate's slow path ran)
            c->tbWide.resize(b->n_tbs);
            uint32_t any = 0;
            for (uint32_t i = 0; i < b->n_tbs; i++) {
                const av1r_tb& t = b->tbs[i];
                uint32_t o = 0;
                for (uint32_t q = 0; q < t.coef_cnt; q++) o |= (cf[t.coef_off + q] + 0x8000u) >> 16;
                c->tbWide[i] = o != 0;
                any |= o;
            }
            c->anyWide = any != 0;
        }
        c->wideKnown = false;  // (one frame's)
        c->nCoef32 = 0;
        if (c->anyWide) {
            c->tbCoefOff.resize(b->n_tbs);
            size_t n32 = 0;
            for (uint32_t i = 0; i < b->n_tbs; i++) {
                c->tbCoefOff[i] = (uint32_t)n32;
                if (c->tbWide[i]) n32 += b->tbs[i].coef_cnt;
            }
            c->nCoef32 = n32;
        }
    } else if (c->anyWide && c->tbWide.size() != b->n_tbs) {
        return fail(c, AV1R_E_INVALID, "pack without its size pass");
    }
    // every coefficient in 16 bits at its own index (a wide TB's there are truncated and
    // unread), the wide TBs' again in 32 bits
    const size_t szCoef = align256(4 * c->nCoef32 + 4);
    const size_t szCoef16 = align256(2 * (size_t)b->n_coefs + 4);
    const size_t szPal = align256(b->n_palette);
    const size_t szCdef = align256((size_t)h->cdef_rows * h->cdef_cols);
    const size_t szLr = align256(sizeof(av1r_lr_unit) * (size_t)b->n_lr_units);
    const size_t szItems = align256(sizeof(WorkItem) * c->items.size() + 4);
    const size_t szTiles = align256(4 * c->tiles.size() + 4);
    const size_t szDeps = align256(4 * c->deps.size() + 4);
    const size_t szDone = align256(4 * c->items.size() + 4);  // zeroed on the device (k_mi_zero): no launch's epoch
    const size_t szTbRes = align256(4 * c->tbRes.size() + 4);
    const size_t szResS = align256(4 * c->residS.size() + 4);
    const size_t szResL = align256(4 * c->residL.size() + 4);
    // the mode-info grid goes last and is not uploaded: k_mi derives it in place
    *need = szHdr + szBlk + szExt + szTb + szCoef + szCoef16 + szPal + szCdef + szLr + szItems + szTiles + szDeps + szTbRes + szResS + szResL + szDone + szMi;
    static const bool sizeDbg = getenv("AV1R_PACK_SIZES") != nullptr;
    if (sizeDbg && host)
    {
        fprintf(stderr, "av1r pack: blocks %zu tbs %zu coefs %zu items %zu (%zu) deps %zu done %zu tbres %zu resid %zu lr %zu levels %zu\n", szBlk,
            szTb, szCoef + szCoef16, szItems, c->items.size(), szDeps, szDone, szTbRes, szResS + szResL, szLr, c->levels.size());
        // k_flow items (large, small) per level: the first levels, then the rest
        uint32_t rest[2] = {};
        for (size_t l = 0; l < c->levels.size(); l++) {
            if (l < 4) fprintf(stderr, "  level %zu: %u large %u small\n", l, c->levels[l].fcnt[1], c->levels[l].fcnt[2]);
            else rest[0] += c->levels[l].fcnt[1], rest[1] += c->levels[l].fcnt[2];
        }
        fprintf(stderr, "  levels 4+: %u large %u small\n", rest[0], rest[1]);
        uint32_t tiny = 0, small = 0;
        for (const Level& lv : c->levels) tiny += lv.tiny, small += lv.fcnt[2];
        fprintf(stderr, "  tiny items %u of %u small k_flow items\n", tiny, small);
    }
    if (!host) return AV1R_OK;
    size_t off = 0;
    // a section of sz bytes at `off`: n bytes copied from src (or, src null, `used` bytes the
    // caller writes in place), the rest of the uploaded sections zeroed -- the packed bytes
    // are a pure function of the frame (no heap contents travel; tests/test_abi.py's digest)
    auto put = [&](const void* src, size_t n, size_t sz, size_t used = 0, bool uploaded = true) {
        if (n) memcpy(host + off, src, n);
        if (uploaded) memset(host + off + (n ? n : used), 0, sz - (n ? n : used));
        size_t o = off;
        off += sz;
        return dev + o;
    };
    KParams& k = P.base;
    memset(&k, 0, sizeof(k));
    k.hdr = (const av1r_frame_hdr*)put(h, sizeof(av1r_frame_hdr), szHdr);
    {
        DevBlock* db = reinterpret_cast<DevBlock*>(host + off);
        k.blocks = (const DevBlock*)put(nullptr, 0, szBlk, sizeof(DevBlock) * (size_t)b->n_blocks);
        int32_t* dx = reinterpret_cast<int32_t*>(host + off);
        k.bext = (const int32_t*)put(nullptr, 0, szExt, 32 * nExt);
        uint32_t w = 0;
        for (uint32_t i = 0; i < b->n_blocks; i++) {
            const av1r_block& s = b->blocks[i];
            DevBlock& d = db[i];
            memcpy(&d, &s, offsetof(DevBlock, palette_off));
            d.palette_off = s.palette_off;
            memcpy(d.mv, s.mv, 16);
            if (s.flags & extFlags) {
                int32_t* e = dx + 8 * (size_t)w;
                memcpy(e, s.local_warp, 24);
                e[6] = (int32_t)s.first_tb;
                e[7] = (int32_t)s.n_tbs;
                d.palette_off = w++;
            }
        }
    }
    {
        // the TBs in the device's record, their coefficients split by width (the size pass's
        // classification)
        DevTb* dt = reinterpret_cast<DevTb*>(host + off);
        k.tbs = (const DevTb*)put(nullptr, 0, szTb, sizeof(DevTb) * (size_t)b->n_tbs);
        uint32_t* c32 = reinterpret_cast<uint32_t*>(host + off);
        k.coefs = (const uint32_t*)put(nullptr, 0, szCoef, 4 * c->nCoef32);
        uint16_t* c16 = reinterpret_cast<uint16_t*>(host + off);
        k.coefs16 = (const uint16_t*)put(nullptr, 0, szCoef16, 2 * (size_t)b->n_coefs);
        for (uint32_t q = 0; q < b->n_coefs; q++) c16[q] = (uint16_t)b->coefs[q];
        for (uint32_t i = 0; i < b->n_tbs; i++) {
            const av1r_tb& t = b->tbs[i];
            const bool wide = c->anyWide && c->tbWide[i];
            DevTb d;  // (composed in registers, stored whole)
            d.block = t.block;
            d.coef_off = wide ? c->tbCoefOff[i] : t.coef_off;
            d.x = t.x;
            d.y = t.y;
            d.coef_cnt = t.coef_cnt;
            d.plane = t.plane;
            d.tx_size = t.tx_size;
            d.tx_type = t.tx_type;
            d.flags = (t.flags & 15u) | (wide ? AV1R_TBD_WIDE : 0u);
            dt[i] = d;
            if (wide) memcpy(c32 + c->tbCoefOff[i], b->coefs + t.coef_off, 4 * (size_t)t.coef_cnt);
        }
    }
    k.palette = put(b->palette, b->n_palette, szPal);
    k.cdef_idx = (const int8_t*)put(b->cdef_idx, (size_t)h->cdef_rows * h->cdef_cols, szCdef);
    k.lr = (const av1r_lr_unit*)put(b->lr_units, sizeof(av1r_lr_unit) * (size_t)b->n_lr_units, szLr);
    static const bool verify = getenv("AV1R_PACK_VERIFY") != nullptr;
    if (verify) {  // (AV1R_PACK_VERIFY, tests/test_abi.py) the device records read back as the kernels read them
        const DevTb* dt = reinterpret_cast<const DevTb*>(host + ((const uint8_t*)k.tbs - dev));
        const uint32_t* c32 = reinterpret_cast<const uint32_t*>(host + ((const uint8_t*)k.coefs - dev));
        const uint16_t* c16 = reinterpret_cast<const uint16_t*>(host + ((const uint8_t*)k.coefs16 - dev));
        for (uint32_t i = 0; i < b->n_tbs; i++) {
            const av1r_tb& t = b->tbs[i];
            const DevTb& d = dt[i];
            if (d.block != t.block || d.x != t.x || d.y != t.y || d.coef_cnt != t.coef_cnt || d.plane != t.plane ||
                d.tx_size != t.tx_size || d.tx_type != t.tx_type || (d.flags & 15u) != t.flags)
                return fail(c, AV1R_E_INVALID, "pack verify: tb %u fields", i);
            for (uint32_t q = 0; q < t.coef_cnt; q++) {
                const uint32_t v = (d.flags & AV1R_TBD_WIDE) ? c32[d.coef_off + q] : (uint32_t)(int32_t)(int16_t)c16[d.coef_off + q];
                if (v != b->coefs[t.coef_off + q]) return fail(c, AV1R_E_INVALID, "pack verify: tb %u coefficient %u", i, q);
            }
        }
    }
    {
        // the items' coefficient references follow their TBs' (offset and width)
        WorkItem* wi = reinterpret_cast<WorkItem*>(host + off);
        P.dItems = (const WorkItem*)put(c->items.data(), sizeof(WorkItem) * c->items.size(), szItems);
        k.items = P.dItems;
        for (size_t i = 0; c->anyWide && i < c->items.size(); i++) {
            const uint32_t code = wi[i].code;
            if (AV1R_ITEM_KIND(code) != AV1R_ITEM_TB) continue;
            const uint32_t ti = AV1R_ITEM_INDEX(code);
            if (!c->tbWide[ti]) continue;
            wi[i].coef_off = c->tbCoefOff[ti];
            wi[i].flags |= AV1R_TBD_WIDE;
        }
        // (the tiny items' slots become TinyItems on the device: k_mi_zero)
    }
    k.tiles = (const uint32_t*)put(c->tiles.data(), 4 * c->tiles.size(), szTiles);
    k.deps = (const uint32_t*)put(c->deps.data(), 4 * c->deps.size(), szDeps);
    k.tb_res = (const uint32_t*)put(c->tbRes.data(), 4 * c->tbRes.size(), szTbRes);
    k.resid_s = (const uint32_t*)put(c->residS.data(), 4 * c->residS.size(), szResS);
    k.resid_l = (const uint32_t*)put(c->residL.data(), 4 * c->residL.size(), szResL);
    P.upBytes = off;  // everything up to here travels; what follows is filled on the device
    k.done = (uint32_t*)put(nullptr, 0, szDone, 0, false);
    k.n_items = (uint32_t)c->items.size();
    k.n_resid_t = c->nResidT;
    k.n_resid_e = c->nResidE;
    k.mi = (const av1r_mi*)put(nullptr, 0, szMi, 0, false);
    if (verify) {
        // every section placed, in order, inside the buffer (a section left out of the
        // packing sequence keeps the null of the memset: below the header's successors)
#define KP_SEC(f) (const void*)k.f,
        const void* secs[] = {AV1R_KP_SECTIONS(KP_SEC)};
#undef KP_SEC
        const uint8_t* prev = dev;
        for (size_t i = 0; i < sizeof(secs) / sizeof(secs[0]); i++) {
            const uint8_t* q = (const uint8_t*)secs[i];
            if (q < prev || (size_t)(q - dev) >= off)  // (empty sections may share an offset)
                return fail(c, AV1R_E_INVALID, "pack verify: section %zu misplaced", i);
            prev = q;
        }
        if (off != *need) return fail(c, AV1R_E_INVALID, "pack verify: %zu bytes packed, %zu sized", off, *need);
    }
    P.flowOk = c->flowOk;
    k.gran = c->flowOk && c->granOk;
    for (int p = 0; p < 3; p++) {
        k.gran_w[p] = c->mapW[p];
        k.gran_hn[p] = c->mapH[p];
    }
    P.nResidS = c->nResidT + c->nResidE + (uint32_t)((c->residS.size() - 64 * c->nResidT - 32 * c->nResidE) / 16);
    P.nResidL = c->nResidM + (uint32_t)(c->residL.size() - 1 - 2 * c->nResidM);
    P.resElems = c->resElems;
    k.mi_stride = h->mi_stride;
    k.mi_cols = h->mi_cols;
    k.mi_rows = h->mi_rows;
    k.mi_rows_alloc = h->mi_rows_alloc;
    k.n_blocks = b->n_blocks;
    k.n_tbs = b->n_tbs;
    k.frame_w = h->frame_width;
    k.frame_h = h->frame_height;
    P.hdr = *h;
    P.levels = c->levels;
    P.bytes = off;
    memcpy(P.usedRef, c->usedRef, sizeof(P.usedRef));
    P.levelsOk = c->levelsOk;
    return AV1R_OK;
}

// ------------------------------------------------------------------------------------
// Launching: a batch of n frames (one per context/stream, n = 1 for the plain API) goes
// through recon -> LF -> CDEF -> LR in shared launches on one HIP stream: every level of
// every frame in one k_level launch, every frame's filters in one launch per filter.
// ------------------------------------------------------------------------------------
struct FrameJob {
    av1r_ctx* c = nullptr;
    const Prepared* P = nullptr;
    KParams k;
    // the frame's buffers R, C, L and their roles: D the deblocked frame, Co the CDEF output,
    // out the frame the frame store and the output queue keep: deblocked in place in R, CDEF
    // into C, LR into L.
    FrameBuf *R = nullptr, *C = nullptr, *L = nullptr;
    FrameBuf *D = nullptr, *Co = nullptr, *out = nullptr;
    bool scaled = false;  // a reference differs in size from the frame (no k_inter_s tiles)
    uint64_t seq = 0;     // the context's frame sequence number
    uint8_t* dev = nullptr;  // P->offsets: the device copy of the packed buffer
};

// resolve references, allocate the frame's buffers, fill its KParams
static int job_begin(FrameJob& j)
{
    av1r_ctx* c = j.c;
    const Prepared& P = *j.P;
    const av1r_frame_hdr* h = &P.hdr;
    for (int r = 1; r < 8; r++) {
        if (!P.usedRef[r]) continue;
        int slot = h->ref_frame_idx[r - 1];
        if (slot < 0 || slot > 7 || !c->slots[slot])
            return fail(c, AV1R_E_INVALID, "reference %d maps to an empty slot", r);
    }
    j.k = P.base;
    j.k.items = P.dItems;
    if (P.offsets) {  // a packed frame: its pointers are offsets into the uploaded buffer
        auto rb = [&](auto& ptr) {
            ptr = reinterpret_cast<std::remove_reference_t<decltype(ptr)>>(j.dev + reinterpret_cast<uintptr_t>(ptr));
        };
#define KP_RB(f) rb(j.k.f);
        AV1R_KP_SECTIONS(KP_RB)
#undef KP_RB
    }
    for (int s = 0; s < 8; s++)
        if (c->slots[s]) j.k.ref[s] = c->slots[s]->d;
    j.scaled = false;
    for (int r = 1; r < 8; r++)
        if (P.usedRef[r]) {
            const DevFrame& f = c->slots[h->ref_frame_idx[r - 1]]->d;
            j.scaled |= f.width != h->frame_width || f.height != h->frame_height;
        }
    j.R = frame_get(c, h->frame_width, h->frame_height);
    j.C = frame_get(c, h->frame_width, h->frame_height);
    j.L = h->uses_lr ? frame_get(c, h->frame_width, h->frame_height) : nullptr;
    if (!j.R || !j.C || (h->uses_lr && !j.L)) return fail(c, AV1R_E_NOMEM, "frame allocation");
    j.k.cur = j.R->d;
    j.D = j.R;
    j.Co = j.C;
    j.out = j.L ? j.L : j.Co;
    if (P.resElems > c->resCap) {
        if (c->resDev) {
            ctx_join(c);
            HIPCHK(hipStreamSynchronize(c->stream));  // in-flight frames may still read it
            (void)hipFree(c->resDev);
            c->resDev = nullptr;
        }
        c->resCap = P.resElems + P.resElems / 4 + 4096;
        HIPCHK(hipMalloc(&c->resDev, 2 * c->resCap));
    }
    j.k.res = c->resDev;
    if (j.k.gran) {
        size_t need = 0;
        for (int p = 0; p < 3; p++) need += 2 * 8 * (size_t)j.k.gran_w[p] * j.k.gran_hn[p];
        if (need > c->granCap) {
            if (c->granDev) {
                ctx_join(c);
                HIPCHK(hipStreamSynchronize(c->stream));
                (void)hipFree(c->granDev);
                c->granDev = nullptr;
            }
            // zeroed (no launch's epoch: epochs start at 1) before any launch can use it:
            // the context's streams are non-blocking, so not behind a null-stream memset
            HIPCHK(hipMalloc(&c->granDev, need));
            HIPCHK(hipMemsetAsync(c->granDev, 0, need, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            c->granCap = need;
        }
        uint64_t* g = c->granDev;
        for (int p = 0; p < 3; p++) {
            const size_t n = (size_t)j.k.gran_w[p] * j.k.gran_hn[p];
            j.k.gran_h[p] = g;
            j.k.gran_v[p] = g + n;
            g += 2 * n;
        }
    }
    j.k.dbk = j.D->d;
    j.k.cdef = j.Co->d;
    if (j.L) j.k.lrout = j.L->d;
    j.seq = ++c->seq;
    return AV1R_OK;
}

// output queue / frame-store refresh (Av1Decoder.cpp:150-153, 111-119)
static void job_end(FrameJob& j)
{
    av1r_ctx* c = j.c;
    const av1r_frame_hdr* h = &j.P->hdr;
    FrameBuf* out = j.out;
    out->seq = j.seq;
    c->lastSeq = j.seq;
    if (h->frame_type == 0 && h->refresh_frame_flags == 0xff) {  // KEY_FRAME refreshing every slot
        std::lock_guard<std::mutex> lock(g_recMu);
        if (c->failed.empty()) c->keySeqs.clear();
        c->keySeqs.push_back(j.seq);
    }
    for (FrameBuf* f : {j.R, j.C, j.L})
        if (f && f != out) frame_unref(c, f);
    if (c->keepStages) {
        frame_ref(out);
        frame_unref(c, c->stage[AV1R_STAGE_LR]);
        c->stage[AV1R_STAGE_LR] = out;
    }
    if (h->show_frame && !c->discardOutput) {
        frame_ref(out);
        c->outq.push_back(out);
    }
    for (int i = 0; i < 8; i++)
        if (h->refresh_frame_flags & (1 << i)) {
            frame_ref(out);
            frame_unref(c, c->slots[i]);
            c->slots[i] = out;
        }
    frame_unref(c, out);
    c->nLevelsLast = (int)j.P->levels.size();
    c->lastUploadBytes = j.P->upBytes;
}

// k_flow launches of different streams may run together: k_flow's workgroups take their
// queues in entry order, so overlapping grids cannot starve each other (recon.hip, k_flow;
// round 1 chained them, each waiting for the previous one): a deep frame (a key frame's long
// intra chain) launched alone on its own stream overlaps the other streams' batches.
// -DAV1R_FLOW_DEBUG: the stream that launched each epoch (av1r_flow_debug classifies the
// overlapping pairs the kernel records as same-stream or cross-stream)
#ifdef AV1R_FLOW_DEBUG
static std::mutex g_epochMu;
static std::vector<std::pair<uint32_t, hipStream_t>> g_epochLog;
static void flow_debug_note(uint32_t epoch, hipStream_t st)
{
    std::lock_guard<std::mutex> lock(g_epochMu);
    g_epochLog.emplace_back(epoch, st);
}
#else
static void flow_debug_note(uint32_t, hipStream_t) {}
#endif

// AV1R_HOST_PROF: host time per phase of launch_jobs, printed when a context is destroyed
struct HostProf {
    double wait = 0, build = 0, launch = 0;
    long calls = 0;
};
static HostProf g_hprof;
static bool host_prof() { static const bool on = getenv("AV1R_HOST_PROF") != nullptr; return on; }
static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static bool deep_frame(const Prepared& P);

// pro: the stream that runs the batch prologue (k_fetch, k_mi), or nullptr for lc's own.
// The packed batches pass their upload stream: the prologue then follows the batch's uploads
// on it and overlaps the stream's previous batch (its filters), and the launch stream waits
// for it once, where it waited for the uploads (av1r_decode_packed_batch).  Only for buffers
// no earlier launch may still use: the packed path's upload ring slots (a prepared frame
// decoded twice in a row would rewrite its mode-info grid under the first decode).
static int launch_jobs(av1r_ctx* lc, std::vector<FrameJob>& jobs, hipStream_t pro = nullptr)
{
    const double tp0 = host_prof() ? now_us() : 0;
    double tp1 = tp0, tp2 = tp0;
    av1r_ctx* c = lc;  // errors are reported on the launching context
    const int n = (int)jobs.size();
    // k_flow workgroups per CU for a deep frame launched by itself (a key frame through the
    // per-frame API; the pipeline's solo frames take 1): fewer idle pollers along its long
    // chain -- a 1080p key frame alone 1.84 ms at the default 8, 1.73 at 4, 1.69 at 3, 1.67
    // at 2 (round 4)
    const int deepPer = 2;
    const int perCU = n == 1 && deep_frame(*jobs[0].P) ? std::min(lc->flowPerCU, deepPer) : lc->flowPerCU;
    if (n > AV1R_MAX_BATCH) return fail(c, AV1R_E_INVALID, "at most %d frames per batch", AV1R_MAX_BATCH);
    ctx_join(lc);
    hipStream_t st = lc->stream;
    int rc;
    // the thread's sticky HIP error may hold the status of an unrelated earlier call (an
    // event query of another launch's record): only this launch's kernels are checked below
    (void)hipGetLastError();
    size_t nLevels = 0;
    int maxUnits = 0, maxMiCols = 0, maxMiRows = 0, maxW = 0, maxH = 0;
    bool anyLr = false;
    for (auto& j : jobs) {
        const av1r_frame_hdr* h = &j.P->hdr;
        nLevels = std::max(nLevels, j.P->levels.size());
        maxUnits = std::max(maxUnits, h->mi_rows * h->mi_cols + 2 * ((h->mi_rows + 1) / 2) * ((h->mi_cols + 1) / 2));
        maxMiCols = std::max(maxMiCols, h->mi_cols);
        maxMiRows = std::max(maxMiRows, h->mi_rows);
        maxW = std::max(maxW, h->frame_width);
        maxH = std::max(maxH, h->frame_height);
        anyLr |= h->uses_lr != 0;
    }
    // launch metadata: [KParams x n][per level: k_inter table (n + 1 prefix counts, n item
    // offsets), k_inter_m and k_inter_s tables (n + 1 group prefix, n offsets, n counts),
    // k_tb table (large prefix, small prefix, large offsets, small offsets)]
    const size_t tabI = 2 * (size_t)n + 1, tabS = 3 * (size_t)n + 1, tabT = 4 * (size_t)n + 2, tabW = tabI + 2 * tabS + tabT;
    const size_t kBytes = align256(sizeof(KParams) * n);
    const size_t tabBytes = align256(4 * tabW * std::max<size_t>(nLevels, 1));
    // k_flow (AV1R_FLOW=0: level launches): every frame's items are flow-schedulable
    bool flow = flow_schedule(lc);
    bool allFlow = true, mustFlow = false;  // flow-only schedules (av1r_pack) run on k_flow
    for (auto& j : jobs) {
        allFlow &= j.P->flowOk;
        mustFlow |= !j.P->levelsOk;
    }
    if (mustFlow && !allFlow) return fail(c, AV1R_E_INVALID, "a flow-only frame batched with a level-schedule frame");
    flow = (flow || mustFlow) && allFlow;
    // k_flow groups: one large item, or up to four small ones
    size_t nGroups = 0;
    for (auto& j : jobs)
        for (const Level& lv : j.P->levels) nGroups += flow_groups(lv);
    const size_t resTabBytes = align256(4 * 2 * ((size_t)n + 1));
    const size_t nEntries = nGroups;
    const size_t need = kBytes + tabBytes + (flow ? FLOW_CTL_BYTES + 8 * nEntries + resTabBytes : 0);
    const bool anyFlow = flow && nEntries;
    Upload& M = lc->meta[lc->metaIdx];
    lc->metaIdx = (lc->metaIdx + 1) % av1r_ctx::kMetaRing;
    if (M.pending) {
        HIPCHK(hipEventSynchronize(M.done));
        if (host_prof()) tp1 = now_us();
        M.pending = false;
        harvest(false);  // device errors reach their frames (av1r_get_output / av1r_synchronize)
    }
    // the launch's status record (k_flow launches only)
    LaunchRec* rec = nullptr;
    if (anyFlow) {
        std::lock_guard<std::mutex> lock(g_recMu);
        if (!g_recFree.empty()) {
            rec = g_recFree.back();
            g_recFree.pop_back();
        }
    }
    if (anyFlow && !rec) {
        rec = new LaunchRec;
        if (hipHostMalloc(&rec->err, 64) != hipSuccess || hipEventCreateWithFlags(&rec->done, hipEventDisableTiming) != hipSuccess) {
            delete rec;
            return fail(c, AV1R_E_NOMEM, "launch record");
        }
        *rec->err = 0;
    }
    if (M.cap < need) {  // (rare: the frees stall the device; sizes are powers of two, >= 1 MiB)
        if (M.host) (void)hipHostFree(M.host);
        if (M.dev) (void)hipFree(M.dev);
        size_t cap = (size_t)1 << 20;
        while (cap < need) cap <<= 1;
        HIPCHK(hipHostMalloc(&M.host, cap));
        HIPCHK(hipMalloc(&M.dev, cap));
        M.cap = cap;
    }
    KParams* hk = reinterpret_cast<KParams*>(M.host);
    uint32_t frameRows = 0;  // k_flow-mode timeline: frame-major rows
    for (int i = 0; i < n; i++) {
        hk[i] = jobs[i].k;
        hk[i].fi = g_fastIntra.load(std::memory_order_relaxed);
        hk[i].trace_base = frameRows;
        for (const Level& lv : jobs[i].P->levels) frameRows += lv.cnt[0] + lv.cnt[1] + lv.cnt[2];
    }
    uint32_t* tab = reinterpret_cast<uint32_t*>(M.host + kBytes);
    // total[l * 5 + kind]: workgroups of the level's k_inter / k_inter_m / k_inter_s
    // launches, items of its large / small TB lists; totalP: its plain inter tiles
    std::vector<uint32_t> total(nLevels * 5, 0), totalP(nLevels, 0);
    for (size_t l = 0; l < nLevels; l++) {
        uint32_t* ti = tab + l * tabW;       // k_inter
        uint32_t* tm = ti + tabI;            // k_inter_m
        uint32_t* ts = tm + tabS;            // k_inter_s
        uint32_t* tt = ts + tabS;            // k_tb
        ti[0] = tm[0] = ts[0] = tt[0] = tt[n + 1] = 0;
        for (int i = 0; i < n; i++) {
            const auto& lv = jobs[i].P->levels;
            const bool has = l < lv.size();
            const bool plain = has && !jobs[i].scaled;
            const uint32_t md = plain ? lv[l].pl[0] : 0, sm = plain ? lv[l].pl[1] : 0;
            const uint32_t rest = has ? lv[l].cnt[0] - md - sm : 0;
            ti[i + 1] = ti[i] + rest;
            ti[n + 1 + i] = has ? lv[l].off[0] : 0;
            tm[i + 1] = tm[i] + (md + 1) / 2;
            tm[n + 1 + i] = has ? lv[l].off[0] + rest : 0;
            tm[2 * n + 1 + i] = md;
            ts[i + 1] = ts[i] + (sm + 3) / 4;
            ts[n + 1 + i] = has ? lv[l].off[0] + rest + md : 0;
            ts[2 * n + 1 + i] = sm;
            totalP[l] += md + sm;
            tt[i + 1] = tt[i] + (has ? lv[l].cnt[1] : 0);
            tt[n + 2 + i] = tt[n + 1 + i] + (has ? lv[l].cnt[2] : 0);
            tt[2 * n + 2 + i] = has ? lv[l].off[1] : 0;
            tt[3 * n + 2 + i] = has ? lv[l].off[2] : 0;
        }
        total[l * 5 + 0] = ti[n];
        total[l * 5 + 1] = tm[n];
        total[l * 5 + 2] = ts[n];
        total[l * 5 + 3] = tt[n];
        total[l * 5 + 4] = tt[2 * n + 1];
    }
    uint32_t* ctl = reinterpret_cast<uint32_t*>(M.dev + kBytes + tabBytes);
    if (flow) {
        // control block (zeroed) + the groups in topological order: level by level, the
        // frames interleaved; {frame << 8 | n, first item}: n = 0 one large item, n | FLOW_G_TINY
        // 1..FLOW_TINY_G tiny items, else 1..flow_small_group() small items
        memset(M.host + kBytes + tabBytes, 0, FLOW_CTL_BYTES);
        uint32_t* hctl = reinterpret_cast<uint32_t*>(M.host + kBytes + tabBytes);
        *reinterpret_cast<uint32_t**>(hctl + FLOW_HOSTERR) = rec ? rec->err : nullptr;
        hctl[FLOW_SPINLIM] = lc->flowSpins;
        uint32_t* g = reinterpret_cast<uint32_t*>(M.host + kBytes + tabBytes + FLOW_CTL_BYTES);
        for (size_t l = 0; l < nLevels; l++)
            for (int i = 0; i < n; i++) {
                const auto& lvs = jobs[i].P->levels;
                if (l >= lvs.size()) continue;
                const Level& lv = lvs[l];
                for (uint32_t q = 0; q < lv.fcnt[1]; q++, g += 2) {
                    g[0] = (uint32_t)i << 8;
                    g[1] = lv.off[1] + q;
                }
                for (uint32_t q = 0; q < lv.tiny; q += FLOW_TINY_G, g += 2) {
                    g[0] = ((uint32_t)i << 8) | FLOW_G_TINY | std::min<uint32_t>(FLOW_TINY_G, lv.tiny - q);
                    g[1] = lv.off[2] + q;
                }
                const uint32_t G = flow_small_group(lv);
                for (uint32_t q = lv.tiny; q < lv.fcnt[2]; q += G, g += 2) {
                    g[0] = ((uint32_t)i << 8) | std::min<uint32_t>(G, lv.fcnt[2] - q);
                    g[1] = lv.off[2] + q;
                }
            }
        // k_resid tables: prefix sums of the frames' workgroup counts (small, large)
        uint32_t* rt = g;
        rt[0] = rt[n + 1] = 0;
        for (int i = 0; i < n; i++) {
            rt[i + 1] = rt[i] + jobs[i].P->nResidS;
            rt[n + 2 + i] = rt[n + 1 + i] + jobs[i].P->nResidL;
        }
    }
    if (host_prof()) tp2 = now_us();
    hipStream_t ps = pro ? pro : st;
    launch_k_fetch(M.dev, M.host, need, ps);
    const uint32_t* dtab = reinterpret_cast<const uint32_t*>(M.dev + kBytes);
    // the frames' KParams head the metadata buffer (read through the constant address space)
    const KParams* dk = reinterpret_cast<const KParams*>(M.dev);
    {  // the frames' mode-info grids, derived on the device from their blocks and TBs
        uint32_t maxUnits = 0, maxBlocks = 0, maxTbs = 0;
        for (auto& j : jobs) {
            maxUnits = std::max({maxUnits, (uint32_t)(j.k.mi_stride * j.k.mi_rows_alloc), j.k.n_items});
            maxBlocks = std::max(maxBlocks, j.k.n_blocks);
            maxTbs = std::max(maxTbs, j.k.n_tbs);
        }
        launch_k_mi(dk, n, maxUnits, maxBlocks, maxTbs, ps);
    }
    if (pro) {
        HIPCHK(hipEventRecord(lc->pkReady, pro));
        HIPCHK(hipStreamWaitEvent(st, lc->pkReady, 0));
    }

    if (lc->timing) {
        if (lc->evUsed == lc->evPool.size()) {
            std::array<hipEvent_t, 7> e;
            for (auto& x : e) HIPCHK(hipEventCreate(&x));
            lc->evPool.push_back(e);
            lc->evFrames.push_back(0);
        }
        for (int i = 0; i < 7; i++) lc->ev[i] = lc->evPool[lc->evUsed][i];
        lc->evFrames[lc->evUsed] = n;
        lc->evUsed++;
        HIPCHK(hipEventRecord(lc->ev[0], st));
    }
    // the single-frame path keeps per-stage snapshots for av1r_read_stage
    const bool snap = n == 1 && lc->keepStages;
    auto snapshot = [&](int stg, FrameBuf* src) -> int {
        const av1r_frame_hdr* h = &jobs[0].P->hdr;
        FrameBuf* s = frame_get(lc, h->frame_width, h->frame_height);
        if (!s) return fail(c, AV1R_E_NOMEM, "stage allocation");
        for (int p = 0; p < 3; p++) launch_k_copy_plane(s->d.pl[p], src->d.pl[p], st);
        frame_unref(lc, lc->stage[stg]);
        lc->stage[stg] = s;
        return AV1R_OK;
    };

    // ---- reconstruction
    size_t allItems = 0;
    for (uint32_t v : total) allItems += v;
    allItems = std::max<size_t>(allItems, frameRows);
    if (lc->traceFile && lc->traceCap < allItems) {
        if (lc->traceDev) (void)hipFree(lc->traceDev);
        lc->traceCap = allItems + allItems / 2;
        HIPCHK(hipMalloc(&lc->traceDev, lc->traceCap * 128));
    }
    unsigned long long* trace = lc->traceFile ? lc->traceDev : nullptr;
    if (trace) HIPCHK(hipMemsetAsync(trace, 0, allItems * 128, st));  // rows of items not run stay 0
    uint32_t traceBase = 0;
    static std::atomic<uint32_t> epochs{0};
    if (flow) {
        // level 0's inter tiles in one grid (k_inter_all: the general, medium and small
        // classes; round 5: three launches 0.058 ms/frame, one 0.049), then every TB /
        // inter-intra item in one dataflow launch.
        // AV1R_INTER_BANDS: each XCD's share walked band by band over the three classes.
        // Measured (profiles/r05_ab_inter_bands.txt, 1080p x 8): 4 bands fetch 22.3 instead of
        // 29.2 MB per frame in the same time (16: 21.8 MB, 4 % slower)
        static const uint32_t nb = getenv("AV1R_INTER_BANDS") ? (uint32_t)std::max(1, std::min(64, atoi(getenv("AV1R_INTER_BANDS")))) : 4u;
        const uint32_t unit = 8 * nb;
        auto pad8 = [unit](uint32_t v) { return (v + unit - 1) / unit * unit; };
        if (total[0] + total[1] + total[2])
            launch_k_inter_all(dk, dtab, n, pad8(total[0]), pad8(total[1]), pad8(total[2]), nb, trace, st);
        if (lc->timing) HIPCHK(hipEventRecord(lc->ev[5], st));
        // every residual (inter TBs outside inter-intra blocks added in place)
        const uint32_t* drt = reinterpret_cast<const uint32_t*>(M.dev + kBytes + tabBytes + FLOW_CTL_BYTES + 8 * nEntries);
        const uint32_t* hrt = reinterpret_cast<const uint32_t*>(M.host + kBytes + tabBytes + FLOW_CTL_BYTES + 8 * nEntries);
        if (hrt[n]) launch_k_resid(0, dk, drt, n, hrt[n], st);
        if (hrt[2 * n + 1]) launch_k_resid(1, dk, drt + n + 1, n, hrt[2 * n + 1], st);
        if (lc->timing) HIPCHK(hipEventRecord(lc->ev[6], st));
        if (nEntries) {
            if (lc->device < 0 || lc->device >= 64) return fail(c, AV1R_E_DEVICE, "device index");
            // the persistent grid: every resident slot (lc->flowPerCU workgroups per CU; a
            // solo deep frame takes one per CU and leaves the rest to concurrent batches)
            const int grid = (int)std::min<size_t>(flow_grid(lc->device, perCU), (nGroups + FLOW_QUEUES - 1) / FLOW_QUEUES * FLOW_QUEUES);
            // (unique per launch)
            uint32_t epoch = ++epochs;
            if (!epoch) epoch = ++epochs;
            launch_k_flow(dk, M.dev + kBytes + tabBytes + FLOW_CTL_BYTES, (uint32_t)nGroups, ctl, rec->err, epoch, grid, trace, st);
            flow_debug_note(epoch, st);
        }
    }
    if (!flow && lc->timing) {
        HIPCHK(hipEventRecord(lc->ev[5], st));
        HIPCHK(hipEventRecord(lc->ev[6], st));
    }
    for (size_t l = 0; l < nLevels && !flow; l++) {
        const uint32_t* lt = dtab + l * tabW;
        const uint32_t nInter = total[l * 5], nLarge = total[l * 5 + 3], nSmall = total[l * 5 + 4];
        if (nInter) launch_k_level(0, dk, lt, n, nInter, trace, traceBase, st);
        if (total[l * 5 + 1]) launch_k_level(2, dk, lt + tabI, n, total[l * 5 + 1], trace, traceBase, st);
        if (total[l * 5 + 2]) launch_k_level(3, dk, lt + tabI + tabS, n, total[l * 5 + 2], trace, traceBase, st);
        traceBase += nInter + totalP[l];  // (k_inter_m / k_inter_s write no timeline rows)
        if (nLarge + nSmall) launch_k_level(1, dk, lt + tabI + 2 * tabS, n, nLarge + (nSmall + 3) / 4, trace, traceBase, st);
        traceBase += nLarge + nSmall;
    }
    if (trace) {
        // rows of 16: code, stream << 32 | tx_size << 8 | pred, t_entry, t_item, t_pred, t_end, level,
        // then sub-phase stamps (TB: 8 edges, 9 predicted, 11 zeroed, 12 dequantised, 13 rows)
        std::vector<unsigned long long> hv((size_t)allItems * 16);
        HIPCHK(hipMemcpyAsync(hv.data(), trace, hv.size() * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (flow) {  // frame-major rows: each frame's items in their level order, then its tiles
            size_t q = 0;
            for (auto& j : jobs) {
                for (size_t l = 0; l < j.P->levels.size(); l++)
                    for (uint32_t i = 0; i < j.P->levels[l].cnt[1] + j.P->levels[l].cnt[2]; i++, q++) hv[q * 16 + 6] = l;
                for (size_t l = 0; l < j.P->levels.size(); l++)
                    for (uint32_t i = 0; i < j.P->levels[l].cnt[0]; i++, q++) hv[q * 16 + 6] = l;
            }
            hv.resize(q * 16);
        } else {
            size_t q = 0;
            for (size_t l = 0; l < nLevels; l++)
                for (uint32_t i = 0; i < total[l * 5] + totalP[l] + total[l * 5 + 3] + total[l * 5 + 4]; i++, q++)
                    hv[q * 16 + 6] = l;
        }
        fwrite(hv.data(), 8, hv.size(), lc->traceFile);
        fflush(lc->traceFile);
    }
    HIPCHK(hipGetLastError());
    if (snap && (rc = snapshot(AV1R_STAGE_RECON, jobs[0].R))) return rc;
    if (lc->timing) HIPCHK(hipEventRecord(lc->ev[1], st));
    // ---- the in-loop filters (decode_frame_wrapup, Av1Decoder.cpp:181-189)
#ifdef AV1R_FUSED_STRIPE
    // (A/B build: the three filters fused per LR stripe, filters.hip k_stripe; without stage
    // snapshots, which need the deblocked and CDEF frames)
    if (!snap) {
        static const int runTiles = getenv("AV1R_STRIPE_RUN") ? std::max(1, atoi(getenv("AV1R_STRIPE_RUN"))) : 8;
        launch_k_stripe(dk, n, maxW, maxH, runTiles, st);
        if (lc->timing) {
            HIPCHK(hipEventRecord(lc->ev[2], st));
            HIPCHK(hipEventRecord(lc->ev[3], st));
            HIPCHK(hipEventRecord(lc->ev[4], st));
        }
        goto filters_done;
    }
#endif
    // deblocking (LoopFilter::filter, LoopFilter.cpp:40-58): in place, one launch per pass
    // (k_lf).  Round 5 measured both passes of a 64x64 tile in LDS into a frame of their own
    // (k_deblock, its edge decisions from a separate k_lfcode launch): 0.0141-0.0147 ms per
    // 1080p frame against k_lf's 0.0108 (profiles/r05_ab_switches.txt); removed in round 6.
    launch_k_lf(dk, n, 0, maxUnits, st);
    launch_k_lf(dk, n, 1, maxUnits, st);
    if (snap && (rc = snapshot(AV1R_STAGE_LF, jobs[0].D))) return rc;
    if (lc->timing) HIPCHK(hipEventRecord(lc->ev[2], st));
    // ---- CDEF into its own frame (Cdef::filter copies the frame, Cdef.cpp:43)
    launch_k_cdef(dk, n, maxMiCols, maxMiRows, st);
    if (snap) {
        frame_ref(jobs[0].Co);
        frame_unref(lc, lc->stage[AV1R_STAGE_CDEF]);
        lc->stage[AV1R_STAGE_CDEF] = jobs[0].Co;
    }
    if (lc->timing) HIPCHK(hipEventRecord(lc->ev[3], st));
    // ---- loop restoration into its own frame (LoopRestoration.cpp:191-219)
    if (anyLr) launch_k_lr(dk, n, maxW, maxH, st);
    if (lc->timing) HIPCHK(hipEventRecord(lc->ev[4], st));
#ifdef AV1R_FUSED_STRIPE
filters_done:
#endif
    HIPCHK(hipGetLastError());
    // the slot's generation moves on only once this launch is certain to record its event
    // (an early return above leaves waiters on the slot's previous launch, which completed)
    M.gen.fetch_add(1, std::memory_order_release);  // (waiters on this slot's previous launch see it finished)
    lc->lastMeta = &M;
    HIPCHK(hipEventRecord(M.done, st));
    M.pending = true;
    const uint64_t gen = M.gen.load(std::memory_order_relaxed);
    for (auto& j : jobs) {
        for (FrameBuf* f : {j.R, j.C, j.L})
            if (f) f->wMeta = &M, f->wGen = gen;
        job_end(j);
    }
    if (rec) {
        rec->meta = &M;
        rec->gen = M.gen.load(std::memory_order_relaxed);
        std::lock_guard<std::mutex> lock(g_recMu);
        for (auto& j : jobs) rec->members.emplace_back(j.c, j.seq);
        g_recPending.push_back(rec);
    }
    if (host_prof()) {
        const double tp3 = now_us();
        g_hprof.wait += (tp1 > tp0 ? tp1 : tp0) - tp0;
        g_hprof.build += tp2 - (tp1 > tp0 ? tp1 : tp0);
        g_hprof.launch += tp3 - tp2;
        g_hprof.calls++;
    }
    return AV1R_OK;
}

// A frame whose dependency chain is long -- a key frame's intra wavefront: ~2 000 levels
// at 1080p against ~80 for an inter frame -- holds a shared batch for its whole chain.  The
// batched entry points launch it alone on its own context's stream instead (k_flow on one
// workgroup per CU), where it overlaps the other streams' batches: frames of more than 400
// levels.  Round 5: kept in the shared batches -12 % device-only, alone on two workgroups per
// CU -2 % (profiles/r05_ab_solo.txt); round 3: on at most 64 workgroups, k_flow +10 % (1080p)
// and +85 % (4K).
static bool deep_frame(const Prepared& P)
{
    return P.flowOk && (int)P.levels.size() > 400;
}

static int launch_solo(FrameJob& j, hipStream_t pro = nullptr)
{
    av1r_ctx* m = j.c;
    av1r_ctx* c = m;
    std::vector<FrameJob> one(1, j);
    // one k_flow workgroup per CU for a solo deep frame
    const int per = m->flowPerCU;
    m->flowPerCU = 1;
    int rc = launch_jobs(m, one, pro);
    m->flowPerCU = per;
    if (rc) return rc;
    HIPCHK(hipEventRecord(m->soloDone, m->stream));
    m->soloPending = true;
    return AV1R_OK;
}

static int launch_frame(av1r_ctx* c, const Prepared& P)
{
    std::vector<FrameJob> jobs(1);
    jobs[0].c = c;
    jobs[0].P = &P;
    int rc = job_begin(jobs[0]);
    if (rc) return rc;
    return launch_jobs(c, jobs);
}

// streaming path: one pinned staging buffer -> one async H2D copy (ring of 2)
static int run_frame(av1r_ctx* c, const av1r_frame_batch* b)
{
    ctx_join(c);
    c->skipSlotCheck = true;  // slot presence is checked at launch time
    int rc = validate(c, b);
    c->skipSlotCheck = false;
    if (rc) return rc;
    // a frame for k_flow is scheduled for it alone (no level lists; tiny items): as av1r_pack
    build_schedule(c, b, true, flow_schedule(c));
    Prepared& P = c->streamP;
    size_t need = 0;
    pack_frame(c, b, P, nullptr, nullptr, &need);
    Upload& U = c->up[c->upIdx];
    c->upIdx ^= 1;
    if (U.pending) {
        HIPCHK(hipEventSynchronize(U.done));
        U.pending = false;
    }
    if (U.cap < need) {
        if (U.host) (void)hipHostFree(U.host);
        if (U.dev) (void)hipFree(U.dev);
        size_t cap = need + need / 2;
        HIPCHK(hipHostMalloc(&U.host, cap));
        HIPCHK(hipMalloc(&U.dev, cap));
        U.cap = cap;
    }
    if (int prc = pack_frame(c, b, P, U.host, U.dev, &need)) return prc;
    HIPCHK(hipMemcpyAsync(U.dev, U.host, P.upBytes, hipMemcpyHostToDevice, c->stream));
    rc = launch_frame(c, P);
    if (rc) return rc;
    HIPCHK(hipEventRecord(U.done, c->stream));
    U.pending = true;
    return AV1R_OK;
}

// ====================================================================================
// C-ABI
// ====================================================================================
extern "C" {

int av1r_create(int device, av1r_ctx** out)
{
    if (!out) return AV1R_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return AV1R_E_DEVICE;
    av1r_ctx* c = new av1r_ctx;
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return AV1R_E_DEVICE;
    }
    for (int i = 0; i < 2; i++) (void)hipEventCreateWithFlags(&c->up[i].done, hipEventDisableTiming);
    for (auto& u : c->pk) (void)hipEventCreateWithFlags(&u.done, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&c->pkReady, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&c->soloDone, hipEventDisableTiming);
    for (auto& m : c->meta) {
        (void)hipEventCreateWithFlags(&m.done, hipEventDisableTiming);
    }
    if (hipStreamCreateWithFlags(&c->copyStream, hipStreamNonBlocking) != hipSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return AV1R_E_DEVICE;
    }
    (void)hipEventCreateWithFlags(&c->sync, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&c->joinEv, hipEventDisableTiming);
    for (int i = 0; i < 7; i++) (void)hipEventCreate(&c->ev[i]);
    c->evPool.reserve(64);
    if (const char* tf = getenv("AV1R_TRACE_FILE")) c->traceFile = fopen(tf, "ab");
    {
        std::lock_guard<std::mutex> lock(g_ctxMu);
        g_ctxs.push_back(c);
    }
    *out = c;
    return AV1R_OK;
}

void av1r_destroy(av1r_ctx* c)
{
    if (!c) return;
    ctx_join(c);
    if (host_prof() && g_hprof.calls) {
        fprintf(stderr, "av1r host: %ld launches, per launch wait %.1f us, build %.1f us, launch %.1f us\n", g_hprof.calls,
            g_hprof.wait / g_hprof.calls, g_hprof.build / g_hprof.calls, g_hprof.launch / g_hprof.calls);
        g_hprof = HostProf();
    }
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->copyStream);
    if (c->outStream) (void)hipStreamSynchronize(c->outStream);
    for (av1r_output_ticket* t : c->tickets) {  // tickets never waited for die with the context
        if (t->ready) (void)hipEventDestroy(t->ready);
        if (t->done) (void)hipEventDestroy(t->done);
        delete t;
    }
    c->tickets.clear();
    for (auto& S : c->staged) c->stageFree.push_back({S.buf, S.cap});
    for (auto& b : c->stageFree) (void)hipHostFree(b.first);
    c->staged.clear();
    c->stageFree.clear();
    if (c->outStream && c->outStream != c->copyStream) (void)hipStreamDestroy(c->outStream);
    {  // members of its batches: their pending join on its (now drained) stream is satisfied
        std::lock_guard<std::mutex> lock(g_ctxMu);
        for (av1r_ctx* m : g_ctxs)
            if (m->joinLead == c) m->joinLead = nullptr;
        g_ctxs.erase(std::remove(g_ctxs.begin(), g_ctxs.end(), c), g_ctxs.end());
        // what waits for a launch through this context's meta slots (other
        // contexts' upload slots, pooled packed buffers, status records) is complete now
        // (its streams are drained): forget the slots before they go
        auto mine = [&](const Upload* m) { return m >= c->meta && m < c->meta + av1r_ctx::kMetaRing; };
        for (av1r_ctx* m : g_ctxs) {
            for (auto& u : m->pk)
                if (u.waitMeta && mine(u.waitMeta)) {
                    u.waitMeta = nullptr;
                    u.pending = false;
                }
            for (av1r_output_ticket* t : m->tickets)
                if (t->readyMeta && mine(t->readyMeta)) t->readyMeta = nullptr;  // (ready: its event was never recorded)
            for (FrameBuf* f : m->pool)
                if (f->wMeta && mine(f->wMeta)) f->wMeta = nullptr;
        }
        {  // every packed buffer: the pooled ones and those still held by their callers
            std::lock_guard<std::mutex> pl(g_packMu);
            for (av1r_packed* q : g_packAll)
                if (q->waitMeta && mine(q->waitMeta)) {
                    q->waitMeta = nullptr;
                    q->copyPending = false;
                }
        }
        harvest(false);
        std::lock_guard<std::mutex> rl(g_recMu);
        for (LaunchRec* r : g_recPending)
            if (r->meta && mine(r->meta)) r->meta = nullptr;  // (its never-recorded event queries complete)
    }
    for (FrameBuf* f : c->pool) {
        (void)hipFree(f->base);
        delete f;
    }
    auto freeUpload = [](Upload& u) {
        if (u.host) (void)hipHostFree(u.host);
        if (u.dev) (void)hipFree(u.dev);
        (void)hipEventDestroy(u.done);
    };
    for (auto& u : c->up) freeUpload(u);
    for (auto& u : c->pk) freeUpload(u);
    for (auto& u : c->meta) freeUpload(u);
    (void)hipStreamSynchronize(c->copyStream);
    (void)hipStreamDestroy(c->copyStream);
    if (c->resDev) (void)hipFree(c->resDev);
    if (c->granDev) (void)hipFree(c->granDev);
    harvest(false);  // records of launches on its (now idle) stream are complete
    {  // the context leaves every launch record still pending
        std::lock_guard<std::mutex> lock(g_recMu);
        for (LaunchRec* r : g_recPending)
            r->members.erase(std::remove_if(r->members.begin(), r->members.end(),
                                 [&](const std::pair<av1r_ctx*, uint64_t>& m) { return m.first == c; }),
                r->members.end());
    }
    (void)hipEventDestroy(c->sync);
    (void)hipEventDestroy(c->joinEv);
    (void)hipEventDestroy(c->pkReady);
    (void)hipEventDestroy(c->soloDone);
    if (c->traceDev) (void)hipFree(c->traceDev);
    if (c->traceFile) fclose(c->traceFile);
    for (auto& e : c->evPool)
        for (auto& x : e) (void)hipEventDestroy(x);
    for (Prepared* P : c->prepared)
        if (P) {
            if (P->dev) (void)hipFree(P->dev);
            delete P;
        }
    (void)hipStreamDestroy(c->stream);
    delete c;
}

int av1r_decode_frame(av1r_ctx* c, const av1r_frame_batch* b)
{
    if (!c || !b || !b->hdr) return AV1R_E_INVALID;
    if (b->hdr->version != AV1R_VERSION) return fail(c, AV1R_E_INVALID, "batch version %u", b->hdr->version);
    (void)hipSetDevice(c->device);
    if (b->hdr->show_existing_frame) return av1r_show_existing(c, b->hdr->frame_to_show, b->hdr->refresh_frame_flags);
    const int rc = run_frame(c, b);
    return rc ? rc : stage_outputs(c);
}

int av1r_frame_begin(av1r_ctx* c, const av1r_frame_batch* f)
{
    if (!c || !f || !f->hdr || !f->mi || !f->cdef_idx) return AV1R_E_INVALID;
    const av1r_frame_hdr* h = f->hdr;
    c->fHdr.assign((const uint8_t*)h, (const uint8_t*)h + sizeof(*h));
    c->fMi.assign(f->mi, f->mi + (size_t)h->mi_stride * h->mi_rows_alloc);
    c->fCdef.assign(f->cdef_idx, f->cdef_idx + (size_t)h->cdef_rows * h->cdef_cols);
    c->fLr.assign(f->lr_units, f->lr_units + f->n_lr_units);
    c->fBlocks.clear();
    c->fTbs.clear();
    c->fCoefs.clear();
    c->fPal.clear();
    c->inFrame = true;
    return AV1R_OK;
}

int av1r_submit_tile(av1r_ctx* c, const av1r_frame_batch* t)
{
    if (!c || !t || !c->inFrame) return AV1R_E_INVALID;
    uint32_t bBase = (uint32_t)c->fBlocks.size(), tBase = (uint32_t)c->fTbs.size();
    uint32_t cBase = (uint32_t)c->fCoefs.size(), pBase = (uint32_t)c->fPal.size();
    for (uint32_t i = 0; i < t->n_blocks; i++) {
        av1r_block b = t->blocks[i];
        b.first_tb += tBase;
        b.palette_off += pBase;
        c->fBlocks.push_back(b);
    }
    for (uint32_t i = 0; i < t->n_tbs; i++) {
        av1r_tb x = t->tbs[i];
        x.block += bBase;
        x.coef_off += cBase;
        c->fTbs.push_back(x);
    }
    c->fCoefs.insert(c->fCoefs.end(), t->coefs, t->coefs + t->n_coefs);
    c->fPal.insert(c->fPal.end(), t->palette, t->palette + t->n_palette);
    return AV1R_OK;
}

int av1r_frame_end(av1r_ctx* c)
{
    if (!c || !c->inFrame) return AV1R_E_INVALID;
    c->inFrame = false;
    av1r_frame_batch b;
    memset(&b, 0, sizeof(b));
    b.hdr = (const av1r_frame_hdr*)c->fHdr.data();
    b.mi = c->fMi.data();
    b.blocks = c->fBlocks.data();
    b.n_blocks = (uint32_t)c->fBlocks.size();
    b.tbs = c->fTbs.data();
    b.n_tbs = (uint32_t)c->fTbs.size();
    b.coefs = c->fCoefs.data();
    b.n_coefs = (uint32_t)c->fCoefs.size();
    b.palette = c->fPal.data();
    b.n_palette = (uint32_t)c->fPal.size();
    b.cdef_idx = c->fCdef.data();
    b.lr_units = c->fLr.data();
    b.n_lr_units = (uint32_t)c->fLr.size();
    return av1r_decode_frame(c, &b);
}

int av1r_prepare(av1r_ctx* c, const av1r_frame_batch* b, int* handle)
{
    if (!c || !b || !b->hdr || !handle) return AV1R_E_INVALID;
    if (b->hdr->version != AV1R_VERSION) return fail(c, AV1R_E_INVALID, "batch version %u", b->hdr->version);
    (void)hipSetDevice(c->device);
    Prepared* P = new Prepared;
    P->hdr = *b->hdr;
    if (!b->hdr->show_existing_frame) {
        c->skipSlotCheck = true;
        int rc = validate(c, b);
        c->skipSlotCheck = false;
        if (rc) {
            delete P;
            return rc;
        }
        build_schedule(c, b, true, flow_schedule(c));
        size_t need = 0;
        pack_frame(c, b, *P, nullptr, nullptr, &need);
        std::vector<uint8_t> host(need);
        if (hipMalloc(&P->dev, need) != hipSuccess) {
            delete P;
            return fail(c, AV1R_E_NOMEM, "prepared batch allocation");
        }
        P->owned = true;
        P->cap = need;
        if (int prc = pack_frame(c, b, *P, host.data(), P->dev, &need)) {
            (void)hipFree(P->dev);
            delete P;
            return prc;
        }
        if (hipMemcpy(P->dev, host.data(), P->upBytes, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(P->dev);
            delete P;
            return fail(c, AV1R_E_DEVICE, "prepared batch upload");
        }
    }
    c->prepared.push_back(P);
    *handle = (int)c->prepared.size() - 1;
    return AV1R_OK;
}

int av1r_decode_prepared(av1r_ctx* c, int handle)
{
    if (!c || handle < 0 || handle >= (int)c->prepared.size() || !c->prepared[handle]) return AV1R_E_INVALID;
    (void)hipSetDevice(c->device);
    const Prepared& P = *c->prepared[handle];
    if (P.hdr.show_existing_frame) return av1r_show_existing(c, P.hdr.frame_to_show, P.hdr.refresh_frame_flags);
    return launch_frame(c, P);
}

int av1r_decode_prepared_batch(av1r_ctx* const* ctxs, const int* handles, int n)
{
    if (!ctxs || !handles || n <= 0) return AV1R_E_INVALID;
    av1r_ctx* lc = ctxs[0];
    if (!lc) return AV1R_E_INVALID;
    for (int i = 0; i < n; i++) {
        av1r_ctx* c = ctxs[i];
        if (!c || c->device != lc->device) return fail(lc, AV1R_E_INVALID, "batch contexts must share one device");
        for (int j = 0; j < i; j++)
            if (ctxs[j] == c) return fail(lc, AV1R_E_INVALID, "a context appears twice in one batch");
        if (handles[i] < 0 || handles[i] >= (int)c->prepared.size() || !c->prepared[handles[i]])
            return fail(lc, AV1R_E_INVALID, "bad prepared handle %d", handles[i]);
    }
    (void)hipSetDevice(lc->device);
    std::vector<FrameJob> jobs;
    jobs.reserve(n);
    for (int i = 0; i < n; i++) {
        const Prepared& P = *ctxs[i]->prepared[handles[i]];
        if (P.hdr.show_existing_frame) {
            int rc = av1r_show_existing(ctxs[i], P.hdr.frame_to_show, P.hdr.refresh_frame_flags);
            if (rc) return rc;
            continue;
        }
        FrameJob j;
        j.c = ctxs[i];
        j.P = &P;
        int rc = job_begin(j);
        if (rc) return rc;
        if (n > 1 && deep_frame(P)) {  // alone on its own stream, overlapping the batch
            if ((rc = launch_solo(j))) return rc;
            continue;
        }
        jobs.push_back(j);
    }
    if (jobs.empty()) return AV1R_OK;
    // one launch on the first member's stream (round 2: sub-batches on their own members'
    // streams, so that one's k_flow tail overlaps another's launches, measured -25 %)
    {
        std::vector<FrameJob>& sub = jobs;
        av1r_ctx* sl = sub[0].c;
        av1r_ctx* c = sl;
        // the launch stream waits for every member's earlier work on its own stream (none
        // if the member's latest work was a batch on this same stream); a member's own
        // stream is ordered after the batch only when it is next used (ctx_join): no
        // cross-queue signal between back-to-back batches
        ctx_join(sl);
        for (auto& j : sub)
            if (j.c != sl && j.c->joinLead != sl) {
                ctx_join(j.c);
                HIPCHK(hipEventRecord(j.c->sync, j.c->stream));
                HIPCHK(hipStreamWaitEvent(sl->stream, j.c->sync, 0));
            }
        int rc = launch_jobs(sl, sub);
        if (rc) return rc;
        for (auto& j : sub)
            if (j.c != sl) j.c->joinLead = sl;
    }
    return AV1R_OK;
}

int av1r_release_prepared(av1r_ctx* c, int handle)
{
    if (!c || handle < 0 || handle >= (int)c->prepared.size() || !c->prepared[handle]) return AV1R_E_INVALID;
    ctx_join(c);
    (void)hipStreamSynchronize(c->stream);
    if (c->prepared[handle]->dev) (void)hipFree(c->prepared[handle]->dev);
    delete c->prepared[handle];
    c->prepared[handle] = nullptr;
    return AV1R_OK;
}

// ---- packed frames: host work off the launching thread ----
static thread_local av1r_ctx t_packScratch;

const char* av1r_pack_last_error(void) { return t_packScratch.err.c_str(); }

// A pooled buffer for a frame of `need` bytes (0: a show-existing entry, no buffer): the
// oldest released one that fits whose upload has completed, else the oldest that fits (its
// upload waited for), else a new one.  Buffers are never freed while the pool is in use --
// hipHostFree / hipHostMalloc cost milliseconds and stall the device and every other
// thread's HIP calls -- and grow in whole MiB with a quarter's margin, so a running pipeline
// stops allocating after its first GOPs.
static std::atomic<int> g_packCount{0};  // packed buffers allocated (pinned host memory)
static av1r_packed* pack_buffer(size_t need)
{
    av1r_packed* pk = nullptr;
    {
        std::lock_guard<std::mutex> lock(g_packMu);
        size_t pick = SIZE_MAX;
        bool idle = false;
        for (size_t i = 0; i < g_packFree.size(); i++) {
            av1r_packed* q = g_packFree[i];
            if (q->cap < need) continue;
            if (pick == SIZE_MAX) pick = i;
            if (!q->copyPending || (q->waitMeta ? meta_done(q->waitMeta, q->waitGen) : !q->copied || hipEventQuery(q->copied) == hipSuccess)) {
                q->copyPending = false;
                pick = i;
                idle = true;
                break;
            }
        }
        // none whose launch has finished: a new buffer rather than a wait, up to a bound (the
        // pool settles at the pipeline's working set during its first GOPs)
        if (!idle && pick != SIZE_MAX && g_packCount.load() < 384) pick = SIZE_MAX;
        if (pick != SIZE_MAX) {
            pk = g_packFree[pick];
            g_packFree.erase(g_packFree.begin() + pick);
        }
    }
    if (pk) {
        if (pk->copyPending) {  // its previous upload may still read the host buffer
            if (pk->waitMeta) meta_wait(pk->waitMeta, pk->waitGen);
            else if (pk->copied) (void)hipEventSynchronize(pk->copied);
            pk->copyPending = false;
        }
        return pk;
    }
    pk = new (std::nothrow) av1r_packed;
    if (!pk) return pk;
    {
        std::lock_guard<std::mutex> lock(g_packMu);
        g_packAll.push_back(pk);
    }
    if (!need) return pk;
    g_packCount++;
    const size_t cap = (need + need / 4 + (1u << 20)) & ~(size_t)((1u << 20) - 1);
    pk->pinned = hipHostMalloc(&pk->host, cap, hipHostMallocDefault) == hipSuccess;
    if (!pk->pinned) pk->host = static_cast<uint8_t*>(malloc(cap));  // no device here (host-only use)
    if (!pk->host) {
        std::lock_guard<std::mutex> lock(g_packMu);
        g_packAll.erase(std::remove(g_packAll.begin(), g_packAll.end(), pk), g_packAll.end());
        delete pk;
        return nullptr;
    }
    pk->cap = cap;
    return pk;
}

int av1r_pack(const av1r_frame_batch* b, av1r_packed** out)
{
    if (!b || !b->hdr || !out) return AV1R_E_INVALID;
    *out = nullptr;
    av1r_ctx* c = &t_packScratch;  // per-thread schedule scratch: av1r_pack is thread-safe
    if (b->hdr->version != AV1R_VERSION) return fail(c, AV1R_E_INVALID, "batch version %u", b->hdr->version);
    if (b->hdr->show_existing_frame) {
        av1r_packed* pk = pack_buffer(0);
        if (!pk) return AV1R_E_NOMEM;
        pk->P = Prepared();
        pk->P.hdr = *b->hdr;
        *out = pk;
        return AV1R_OK;
    }
    c->skipSlotCheck = true;
    PackClock clk;
    int rc = validate(c, b);
    clk.lap(PP_VALIDATE);
    c->skipSlotCheck = false;
    if (rc) return rc;
    build_schedule(c, b, true, true);
    clk = PackClock();
    Prepared tmp;
    size_t need = 0;
    pack_frame(c, b, tmp, nullptr, nullptr, &need);  // the size only (P untouched)
    av1r_packed* pk = pack_buffer(need);
    if (!pk) return AV1R_E_NOMEM;
    Prepared& P = pk->P;
    P = Prepared();
    P.hdr = *b->hdr;
    if (int prc = pack_frame(c, b, P, pk->host, nullptr, &need)) {
        av1r_packed_free(pk);
        return prc;
    }
    clk.lap(PP_COPY);
    if (g_packProf) g_packNs[PP_N]++;
    P.cap = need;
    P.offsets = true;
    *out = pk;
    return AV1R_OK;
}

int av1r_pack_profile(uint64_t* ns, int n, int reset)
{
    const int m = n < PP_N + 1 ? n : PP_N + 1;
    for (int i = 0; i < m && ns; i++) ns[i] = g_packNs[i].load();
    if (reset)
        for (auto& v : g_packNs) v = 0;
    return g_packProf ? PP_N : 0;
}

void av1r_packed_free(av1r_packed* pk)
{
    if (!pk) return;
    std::lock_guard<std::mutex> lock(g_packMu);
    g_packFree.push_back(pk);
}

size_t av1r_packed_bytes(const av1r_packed* pk) { return pk ? pk->P.upBytes : 0; }

const void* av1r_packed_data(const av1r_packed* pk, size_t* bytes)
{
    if (!pk) return nullptr;
    if (bytes) *bytes = pk->P.upBytes;
    return pk->host;
}

// AV1R_PIPE_PROF=1: where av1r_decode_packed_batch spends the launcher's time (seconds,
// summed; printed by av1r_pipeline_run): waiting for an upload slot (the GPU three frames
// behind on that stream), the solo launches, the shared launches, the rest
struct PipeProf {
    double slotWait = 0, solo = 0, shared = 0, total = 0;
    long batches = 0, frames = 0, soloFrames = 0;
};
static PipeProf g_pprof;
static std::mutex g_pprofMu;  // av1r_decode_packed_batch may run on several threads at once
static const bool g_pipeProf = getenv("AV1R_PIPE_PROF") && atoi(getenv("AV1R_PIPE_PROF")) != 0;
static double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
extern "C" void av1r_pipe_prof_dump(double elapsed)
{
    if (!g_pipeProf) return;
    std::lock_guard<std::mutex> lock(g_pprofMu);
    const PipeProf& P = g_pprof;
    fprintf(stderr, "av1r pipe: %.1f ms elapsed, %ld batches (%.2f frames each, %ld solo), launcher: slot wait %.1f ms, "
            "solo launches %.1f ms, shared launches %.1f ms, other %.1f ms\n", 1e3 * elapsed, P.batches,
            P.batches ? (double)P.frames / P.batches : 0.0, P.soloFrames, 1e3 * P.slotWait, 1e3 * P.solo, 1e3 * P.shared,
            1e3 * (P.total - P.slotWait - P.solo - P.shared));
    g_pprof = PipeProf();
}

int av1r_decode_packed_batch(av1r_ctx* const* ctxs, av1r_packed* const* pks, int n)
{
    const double tIn = g_pipeProf ? now_s() : 0;
    struct Tot {
        double t;
        ~Tot()
        {
            if (!g_pipeProf) return;
            std::lock_guard<std::mutex> lock(g_pprofMu);
            g_pprof.total += now_s() - t;
        }
    } tot{tIn};
    if (!ctxs || !pks || n <= 0 || !ctxs[0]) return AV1R_E_INVALID;
    av1r_ctx* lc = ctxs[0];
    av1r_ctx* c = lc;
    for (int i = 0; i < n; i++) {
        if (!ctxs[i] || ctxs[i]->device != lc->device || !pks[i]) return fail(lc, AV1R_E_INVALID, "bad batch member %d", i);
        for (int j = 0; j < i; j++)
            if (ctxs[j] == ctxs[i]) return fail(lc, AV1R_E_INVALID, "a context appears twice in one batch");
    }
    (void)hipSetDevice(lc->device);
    // deep frames go alone on their own context's stream; the rest share launches on the
    // first shallow member's stream
    av1r_ctx* bl = nullptr;
    for (int i = 0; i < n && !bl; i++)
        if (!pks[i]->P.hdr.show_existing_frame && !(n > 1 && deep_frame(pks[i]->P))) bl = ctxs[i];
    if (bl) ctx_join(bl);
    std::vector<FrameJob> jobs, solo;
    std::vector<Upload*> slots(n, nullptr);
    std::vector<bool> metaWait(n, false);  // packed buffers released by the launch's completion
    bool copies = false;
    for (int i = 0; i < n; i++) {
        av1r_ctx* m = ctxs[i];
        av1r_packed* pk = pks[i];
        if (pk->P.hdr.show_existing_frame) {
            int rc = av1r_show_existing(m, pk->P.hdr.frame_to_show, pk->P.hdr.refresh_frame_flags);
            if (rc) return rc;
            continue;
        }
        const bool alone = n > 1 && deep_frame(pk->P);
        // whose copy stream carries the upload: the batch lead's (round 2: every member's own,
        // spreading a batch's copies over the copy engines, measured slower -- 2 834 vs 3 179
        // frames/s host-inclusive)
        av1r_ctx* up = alone ? m : bl;
        Upload& U = m->pk[m->pkIdx];
        slots[i] = &U;
        m->pkIdx = (m->pkIdx + 1) % av1r_ctx::kPackRing;
        if (U.pending) {  // a launch three frames back may still read this slot
            const double w0 = g_pipeProf ? now_s() : 0;
            if (!U.waitMeta) HIPCHK(hipEventSynchronize(U.done));
            else if (U.waitMeta->gen == U.waitGen) HIPCHK(hipEventSynchronize(U.waitMeta->done));
            // (else that meta slot was reused: its launch was waited for then)
            if (g_pipeProf) {
                std::lock_guard<std::mutex> lock(g_pprofMu);
                g_pprof.slotWait += now_s() - w0;
            }
            U.pending = false;
        }
        if (U.cap < pk->P.cap) {
            if (U.dev) (void)hipFree(U.dev);
            U.cap = (pk->P.cap + pk->P.cap / 4 + (1u << 20)) & ~(size_t)((1u << 20) - 1);
            HIPCHK(hipMalloc(&U.dev, U.cap));
        }
        HIPCHK(hipMemcpyAsync(U.dev, pk->host, pk->P.upBytes, hipMemcpyHostToDevice, up->copyStream));
        // the host buffer is free once the upload has landed: an event for a frame launched
        // alone or uploaded on another stream (something waits for it), else its launch's
        // completion (set below)
        pk->waitMeta = nullptr;
        if (alone) {
            if (!pk->copied) HIPCHK(hipEventCreateWithFlags(&pk->copied, hipEventDisableTiming));
            HIPCHK(hipEventRecord(pk->copied, up->copyStream));
        } else {
            metaWait[i] = true;
        }
        pk->copyPending = true;
        if (alone) {
            ctx_join(m);
            HIPCHK(hipStreamWaitEvent(m->stream, pk->copied, 0));
        } else {
            copies = true;
        }
        FrameJob j;
        j.c = m;
        j.P = &pk->P;
        j.dev = U.dev;
        int rc = job_begin(j);
        if (rc) return rc;
        (alone ? solo : jobs).push_back(j);
    }
    const double s0 = g_pipeProf ? now_s() : 0;
    for (auto& j : solo) {  // first, so that their long chains start at once
        int rc = launch_solo(j, j.c->copyStream);  // (its upload went on that stream)
        if (rc) return rc;
    }
    const double s1 = g_pipeProf ? now_s() : 0;
    if (g_pipeProf) {
        std::lock_guard<std::mutex> lock(g_pprofMu);
        g_pprof.solo += s1 - s0;
        g_pprof.batches++;
        g_pprof.frames += n;
        g_pprof.soloFrames += (long)solo.size();
    }
    if (!jobs.empty()) {
        // members' own earlier work first (as av1r_decode_prepared_batch)
        for (auto& j : jobs)
            if (j.c != bl && j.c->joinLead != bl) {
                ctx_join(j.c);
                HIPCHK(hipEventRecord(j.c->sync, j.c->stream));
                HIPCHK(hipStreamWaitEvent(bl->stream, j.c->sync, 0));
            }
        // (the uploads on bl's copy stream: launch_jobs runs the prologue after them there,
        // and bl's stream waits for that)
        (void)copies;
        // a flow-only frame and a level-schedule frame (intra block copy) cannot share launches
        std::vector<FrameJob> lv;
        for (size_t i = 0; i < jobs.size();)
            if (!jobs[i].P->flowOk) {
                lv.push_back(jobs[i]);
                jobs.erase(jobs.begin() + i);
            } else {
                i++;
            }
        int rc = jobs.empty() ? AV1R_OK : launch_jobs(bl, jobs, bl->copyStream);
        if (!rc && !lv.empty()) rc = launch_jobs(bl, lv, bl->copyStream);
        if (rc) return rc;
        for (auto& j : jobs)
            if (j.c != bl) j.c->joinLead = bl;
        for (auto& j : lv)
            if (j.c != bl) j.c->joinLead = bl;
        if (g_pipeProf) {
            std::lock_guard<std::mutex> lock(g_pprofMu);
            g_pprof.shared += now_s() - s1;
        }
    }
    // the upload slots (and the packed buffers) are free again after their launch: its own
    // completion event, through the launch's metadata slot (round 4: an event recorded per
    // slot, per packed buffer and per status record, each a marker packet in the compute
    // stream's hardware queue, held the headline at 6 100 against 6 370 frames/s)
    for (int i = 0; i < n; i++) {
        if (!slots[i]) continue;
        av1r_ctx* m = ctxs[i];
        const bool alone = std::any_of(solo.begin(), solo.end(), [&](const FrameJob& j) { return j.c == m; });
        const Upload* lm = (alone ? m : bl)->lastMeta;
        if (metaWait[i]) {
            pks[i]->waitMeta = bl->lastMeta;
            pks[i]->waitGen = bl->lastMeta ? bl->lastMeta->gen.load(std::memory_order_relaxed) : 0;
            if (!bl->lastMeta) pks[i]->copyPending = false;  // (no launch read it: nothing to wait for)
        }
        if (lm) {
            slots[i]->waitMeta = lm;
            slots[i]->waitGen = lm->gen.load(std::memory_order_relaxed);
        } else {
            slots[i]->waitMeta = nullptr;
            HIPCHK(hipEventRecord(slots[i]->done, alone ? m->stream : bl->stream));
        }
        slots[i]->pending = true;
    }
    return AV1R_OK;
}

// 1 while a deep frame this context launched alone (batched entry points) is running
int av1r_busy(av1r_ctx* c)
{
    if (!c) return AV1R_E_INVALID;
    if (!c->soloPending) return 0;
    if (hipEventQuery(c->soloDone) == hipErrorNotReady) return 1;
    c->soloPending = false;
    return 0;
}

int av1r_set_discard_output(av1r_ctx* c, int discard)
{
    if (!c) return AV1R_E_INVALID;
    c->discardOutput = discard != 0;
    return AV1R_OK;
}

int av1r_show_existing(av1r_ctx* c, int slot, int refresh)
{
    if (!c || slot < 0 || slot > 7 || !c->slots[slot]) return AV1R_E_INVALID;
    ctx_join(c);
    FrameBuf* f = c->slots[slot];
    frame_ref(f);  // hold across the refresh
    frame_ref(f);
    if (!c->discardOutput) c->outq.push_back(f);
    else frame_unref(c, f);
    for (int i = 0; i < 8; i++)
        if (refresh & (1 << i)) {
            frame_ref(f);
            frame_unref(c, c->slots[i]);
            c->slots[i] = f;
        }
    frame_unref(c, f);
    return stage_outputs(c);
}

int av1r_ref_release(av1r_ctx* c, int slotMask)
{
    if (!c || (slotMask & ~0xff)) return AV1R_E_INVALID;
    ctx_join(c);  // (as show_existing: a buffer reused later is written behind the queued reads, in stream order)
    for (int i = 0; i < 8; i++)
        if (slotMask & (1 << i)) {
            frame_unref(c, c->slots[i]);
            c->slots[i] = nullptr;
        }
    return AV1R_OK;
}

int av1r_set_strip_levels(int) { return 0; }
int av1r_set_filter_fusion(int) { return 0; }
int av1r_set_flow_wave(int) { return 0; }

int av1r_output_pending(av1r_ctx* c) { return c ? (int)(c->outq.size() + c->staged.size()) : 0; }

static int copy_plane_d2h(av1r_ctx* c, const DevPlane& p, uint8_t* dst, int ds)
{
    HIPCHK(hipMemcpy2DAsync(dst, ds, p.p, p.stride, p.w, p.h, hipMemcpyDeviceToHost, c->stream));
    return AV1R_OK;
}

static int get_staged(av1r_ctx* c, uint8_t* y, int ys, uint8_t* u, int us, uint8_t* v, int vs, int* width, int* height);

int av1r_get_output(av1r_ctx* c, uint8_t* y, int ys, uint8_t* u, int us, uint8_t* v, int vs, int* width, int* height)
{
    if (!c) return AV1R_E_INVALID;
    if (!c->staged.empty()) return get_staged(c, y, ys, u, us, v, vs, width, height);
    if (c->outq.empty()) return AV1R_E_NO_OUTPUT;
    FrameBuf* f = c->outq.front();
    if (width) *width = f->d.width;
    if (height) *height = f->d.height;
    if (!y) return AV1R_OK;  // the size only: host state, no join of the context's stream
    ctx_join(c);
    (void)hipSetDevice(c->device);
    int rc;
    if ((rc = copy_plane_d2h(c, f->d.pl[0], y, ys)) || (rc = copy_plane_d2h(c, f->d.pl[1], u, us)) || (rc = copy_plane_d2h(c, f->d.pl[2], v, vs)))
        return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    c->outq.pop_front();
    frame_unref(c, f);
    harvest(false);
    std::lock_guard<std::mutex> lock(g_recMu);
    if (frame_failed(c, f->seq)) return fail(c, AV1R_E_DEVICE, "frame %llu: %s", (unsigned long long)f->seq, c->err.c_str());
    return AV1R_OK;
}

static int output_ticket(av1r_ctx* c, uint8_t* y, int ys, uint8_t* u, int us, uint8_t* v, int vs, int* width, int* height,
                         av1r_output_ticket** out, bool needEvent = false);

// No completion event after a read-back: an event recorded on the read-back stream is a
// barrier packet in whichever hardware queue the stream shares with others, holding them
// until the copy is done.  A read-back counts as landed once its stream has gone idle
// (copies on a stream complete in order): the bench's delivery leg 0.96x of the
// undelivered rate against 0.88-0.90x with an event per read-back (round 4).  (A 4-byte
// copy of a flag word after the planes instead of the event measured 0.59x.)

static int ticket_issue(av1r_output_ticket* t, bool event = false);

int av1r_get_output_async(av1r_ctx* c, uint8_t* y, int ys, uint8_t* u, int us, uint8_t* v, int vs, int* width, int* height,
                          av1r_output_ticket** out)
{
    if (!c || !out || !y || !u || !v) return AV1R_E_INVALID;
    *out = nullptr;
    // (the staged frames are older than the queued ones: they must leave first, through
    // av1r_get_output)
    if (!c->staged.empty()) return fail(c, AV1R_E_INVALID, "frames already staged by av1r_set_output_prefetch: use av1r_get_output");
    // (round 4: the copies queued at once behind a device-side wait for the frame, instead
    // of when the host sees it done, measured 0.48x of the undelivered rate)
    return output_ticket(c, y, ys, u, us, v, vs, width, height, out);
}

// the oldest queued frame into a ticket (av1r_get_output_async; stage_outputs)
static int output_ticket(av1r_ctx* c, uint8_t* y, int ys, uint8_t* u, int us, uint8_t* v, int vs, int* width, int* height,
                         av1r_output_ticket** out, bool needEvent)
{
    *out = nullptr;
    if (c->outq.empty()) return AV1R_E_NO_OUTPUT;
    (void)hipSetDevice(c->device);
    if (!c->outStream) {
        // The read-backs go on the context's upload stream (round 4 measured a stream of their
        // own, also one created with a full CU mask: 0.84x).  Each read-back's completion marker sits in whichever of the runtime's
        // 4 hardware queues its stream landed on (streams attach to the least-used queue at
        // creation), holding back the streams that share it.  A stream of their own, created
        // late, shares a queue with a compute stream; the upload stream's queue holds copy
        // streams, but the context's own uploads (a batch lead's, a key frame's) queue
        // behind its read-backs.  Which costs more depends on the streams created before:
        // the bench's delivery leg (after its other legs) 0.89-0.92x of the undelivered rate
        // on the upload stream against 0.82-0.84x on their own; tools/out_probe.py (fresh
        // contexts) the other way round, 0.82x against 0.89x
        c->outStream = c->copyStream;
    }
    av1r_output_ticket* t = nullptr;
    for (av1r_output_ticket* q : c->tickets)
        if (!q->live) {
            t = q;
            break;
        }
    if (!t) {
        t = new (std::nothrow) av1r_output_ticket;
        if (!t) return AV1R_E_NOMEM;
        if (hipEventCreateWithFlags(&t->ready, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&t->done, hipEventDisableTiming) != hipSuccess) {
            if (t->ready) (void)hipEventDestroy(t->ready);
            delete t;
            return fail(c, AV1R_E_DEVICE, "hipEventCreate");
        }
        c->tickets.push_back(t);
    }
    FrameBuf* f = c->outq.front();
    // the frame's last writer: this context's own stream, or the stream of the batch it was
    // last launched in (ctx_join is not needed: nothing is enqueued on the context here)
    // the last launch on that stream has it (members join a batch stream behind their own
    // stream's work, ctx_join): its completion, or an event where a stream must wait on it
    // (the frame's own launch: a show-existing frame, or a context joined since -- ctx_join
    // clears joinLead without enqueuing work -- is not the context's last launch)
    av1r_ctx* w = c->joinLead ? c->joinLead : c;
    t->readyMeta = nullptr;
    if (!needEvent && f->wMeta) {
        t->readyMeta = f->wMeta;
        t->readyGen = f->wGen;
    } else {
        HIPCHK(hipEventRecord(t->ready, w->stream));
    }
    c->outq.pop_front();  // the queue's reference passes to the ticket
    t->c = c;
    t->f = f;
    t->dst[0] = y, t->dst[1] = u, t->dst[2] = v;
    t->ds[0] = ys, t->ds[1] = us, t->ds[2] = vs;
    t->state = 0;
    t->live = true;
    if (width) *width = f->d.width;
    if (height) *height = f->d.height;
    *out = t;
    return AV1R_OK;
}

// event: record the read-back's own completion instead of watching its stream go idle --
// for a copy queued behind a device-side wait (prefetch staging), whose stream also carries
// every later frame's wait and copy
static int ticket_issue(av1r_output_ticket* t, bool event)
{
    av1r_ctx* c = t->c;
    // How the planes travel: on the read-back stream (copy engine), one linear transfer or
    // three 2-D ones.  Round 4 measured a kernel (k_out) storing them straight over the bus
    // into pinned memory: the bus writes slowed every filter kernel 20-40% (8 x 1080p: 0.72x
    // of the undelivered rate against 0.89x); packing them into device staging for one linear
    // copy 0.55x (a kernel on the read-back stream stalls the compute stream sharing its
    // queue).  k_out was removed in round 6.
    const DevPlane* pl = t->f->d.pl;
    const uint8_t* src[3] = {pl[0].p, pl[1].p, pl[2].p};
    const int ss[3] = {pl[0].stride, pl[1].stride, pl[2].stride};
    const int w[3] = {pl[0].w, pl[1].w, pl[2].w}, h[3] = {pl[0].h, pl[1].h, pl[2].h};
    const bool sameLayout = t->dst[1] - t->dst[0] == src[1] - src[0] && t->dst[2] - t->dst[0] == src[2] - src[0] &&
                            t->ds[0] == ss[0] && t->ds[1] == ss[1] && t->ds[2] == ss[2];
    if (sameLayout) {
        // a destination in the library's own layout (av1r_frame_layout; the ring sink): the
        // frame in ONE linear transfer, padding included (three 2-D copies left the copy
        // engine idle between them, ~10 us each)
        const size_t span = (size_t)(src[2] - src[0]) + (size_t)ss[2] * (h[2] - 1) + w[2];
        HIPCHK(hipMemcpyAsync(t->dst[0], src[0], span, hipMemcpyDeviceToHost, c->outStream));
    } else {
        for (int p = 0; p < 3; p++)
            HIPCHK(hipMemcpy2DAsync(t->dst[p], t->ds[p], src[p], ss[p], w[p], h[p], hipMemcpyDeviceToHost, c->outStream));
    }
    t->sq = !event;
    if (!t->sq) HIPCHK(hipEventRecord(t->done, c->outStream));
    t->state = 1;
    return AV1R_OK;
}

int av1r_output_query(av1r_output_ticket* t)
{
    if (!t || !t->live) return AV1R_E_INVALID;
    av1r_ctx* c = t->c;
    (void)hipSetDevice(c->device);
    if (t->state == 0) {
        if (t->readyMeta) {
            if (!meta_done(t->readyMeta, t->readyGen)) return 0;
        } else {
            const hipError_t q = hipEventQuery(t->ready);
            if (q == hipErrorNotReady) return 0;
            if (q != hipSuccess) return fail(c, AV1R_E_DEVICE, "output: %s", hipGetErrorString(q));
        }
        const int rc = ticket_issue(t);
        if (rc) return rc;
    }
    if (t->state == 1) {
        if (t->sq) {
            const hipError_t q = hipStreamQuery(c->outStream);
            if (q == hipErrorNotReady) return 0;
            if (q != hipSuccess) return fail(c, AV1R_E_DEVICE, "output copy: %s", hipGetErrorString(q));
        } else {
            const hipError_t q = hipEventQuery(t->done);
            if (q == hipErrorNotReady) return 0;
            if (q != hipSuccess) return fail(c, AV1R_E_DEVICE, "output copy: %s", hipGetErrorString(q));
        }
        t->state = 2;
    }
    return 1;
}

int av1r_output_start(av1r_output_ticket* t)
{
    if (!t || !t->live) return AV1R_E_INVALID;
    if (t->state) return 1;
    av1r_ctx* c = t->c;
    (void)hipSetDevice(c->device);
    if (t->readyMeta) {
        if (!meta_done(t->readyMeta, t->readyGen)) return 0;
        const int rc = ticket_issue(t);
        return rc ? rc : 1;
    }
    const hipError_t q = hipEventQuery(t->ready);
    if (q == hipErrorNotReady) return 0;
    if (q != hipSuccess) return fail(c, AV1R_E_DEVICE, "output: %s", hipGetErrorString(q));
    const int rc = ticket_issue(t);
    return rc ? rc : 1;
}

int av1r_output_wait(av1r_output_ticket* t)
{
    if (!t || !t->live) return AV1R_E_INVALID;
    av1r_ctx* c = t->c;
    (void)hipSetDevice(c->device);
    int rc = AV1R_OK;
    if (t->state == 0) {
        if (t->readyMeta) meta_wait(t->readyMeta, t->readyGen);
        else if (hipEventSynchronize(t->ready) != hipSuccess) rc = fail(c, AV1R_E_DEVICE, "output: frame wait failed");
        if (!rc) rc = ticket_issue(t);
    }
    if (!rc && t->state == 1) {
        if (t->sq) {
            if (hipStreamSynchronize(c->outStream) != hipSuccess) rc = fail(c, AV1R_E_DEVICE, "output copy wait failed");
        } else if (hipEventSynchronize(t->done) != hipSuccess) {
            rc = fail(c, AV1R_E_DEVICE, "output copy wait failed");
        }
        t->state = 2;
    }
    if (t->state != 2) {
        // a copy may still be in flight: keep the frame out of the pool until the stream is idle
        (void)hipStreamSynchronize(c->outStream);
    }
    FrameBuf* f = t->f;
    frame_unref(c, f);
    t->f = nullptr;
    t->live = false;
    if (rc) return rc;
    harvest(false);
    std::lock_guard<std::mutex> lock(g_recMu);
    if (frame_failed(c, f->seq)) return fail(c, AV1R_E_DEVICE, "frame %llu: %s", (unsigned long long)f->seq, c->err.c_str());
    return AV1R_OK;
}

// av1r_set_output_prefetch: start the read-back of every queued frame into staging buffers
static int stage_outputs(av1r_ctx* c)
{
    while (c->prefetch && !c->outq.empty()) {
        FrameBuf* f = c->outq.front();
        const int w = f->d.width, h = f->d.height, cw = (w + 1) >> 1, ch = (h + 1) >> 1;
        const size_t need = (size_t)w * h + 2 * (size_t)cw * ch;
        av1r_ctx::Staged S{nullptr, nullptr, 0, w, h};
        for (size_t i = 0; i < c->stageFree.size(); i++)
            if (c->stageFree[i].second >= need) {
                S.buf = c->stageFree[i].first;
                S.cap = c->stageFree[i].second;
                c->stageFree.erase(c->stageFree.begin() + i);
                break;
            }
        if (!S.buf) {
            (void)hipSetDevice(c->device);
            if (hipHostMalloc((void**)&S.buf, need, 0) != hipSuccess) return fail(c, AV1R_E_NOMEM, "staging buffer");
            S.cap = need;
        }
        uint8_t* u = S.buf + (size_t)w * h;
        int rc = output_ticket(c, S.buf, w, u, cw, u + (size_t)cw * ch, cw, nullptr, nullptr, &S.t, true);
        if (!rc && hipStreamWaitEvent(c->outStream, S.t->ready, 0) != hipSuccess) rc = fail(c, AV1R_E_DEVICE, "output stream wait");
        if (!rc) rc = ticket_issue(S.t, true);
        if (rc) {
            if (S.t) (void)av1r_output_wait(S.t);
            c->stageFree.push_back({S.buf, S.cap});
            return rc;
        }
        c->staged.push_back(S);
    }
    return AV1R_OK;
}

static int get_staged(av1r_ctx* c, uint8_t* y, int ys, uint8_t* u, int us, uint8_t* v, int vs, int* width, int* height)
{
    av1r_ctx::Staged S = c->staged.front();
    if (width) *width = S.w;
    if (height) *height = S.h;
    if (!y) return AV1R_OK;
    c->staged.pop_front();
    const int rc = av1r_output_wait(S.t);
    const int cw = (S.w + 1) >> 1, ch = (S.h + 1) >> 1;
    const uint8_t* src = S.buf;
    for (int r = 0; r < S.h; r++) memcpy(y + (size_t)r * ys, src + (size_t)r * S.w, S.w);
    src += (size_t)S.w * S.h;
    for (int r = 0; r < ch; r++) memcpy(u + (size_t)r * us, src + (size_t)r * cw, cw);
    src += (size_t)cw * ch;
    for (int r = 0; r < ch; r++) memcpy(v + (size_t)r * vs, src + (size_t)r * cw, cw);
    c->stageFree.push_back({S.buf, S.cap});
    return rc;
}

int av1r_set_output_prefetch(av1r_ctx* c, int on)
{
    if (!c) return AV1R_E_INVALID;
    c->prefetch = on != 0;
    return stage_outputs(c);
}

int av1r_read_stage(av1r_ctx* c, int stage, int plane, uint8_t* dst, int ds)
{
    if (!c || stage < 0 || stage > 3 || plane < 0 || plane > 2 || !c->stage[stage]) return AV1R_E_INVALID;
    (void)hipSetDevice(c->device);
    ctx_join(c);
    int rc = copy_plane_d2h(c, c->stage[stage]->d.pl[plane], dst, ds);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    harvest(false);
    std::lock_guard<std::mutex> lock(g_recMu);
    if (frame_failed(c, c->lastSeq)) return fail(c, AV1R_E_DEVICE, "stage read: %s", c->err.c_str());
    return AV1R_OK;
}

// Waits for the context's work; AV1R_E_DEVICE once for every failure (a k_flow wait that
// timed out in a launch holding one of its frames) not reported by an earlier call.
int av1r_synchronize(av1r_ctx* c)
{
    if (!c) return AV1R_E_INVALID;
    ctx_join(c);
    HIPCHK(hipStreamSynchronize(c->stream));
    harvest(false);
    std::lock_guard<std::mutex> lock(g_recMu);
    if (c->failed.size() > c->failedReported) {
        c->failedReported = c->failed.size();
        return fail(c, AV1R_E_DEVICE, "%s", c->err.c_str());
    }
    return AV1R_OK;
}

int av1r_set_flow_spins(av1r_ctx* c, uint32_t spins)
{
    if (!c) return AV1R_E_INVALID;
    c->flowSpins = spins;
    return AV1R_OK;
}



int av1r_set_fast_intra(int on) { return g_fastIntra.exchange(on ? 1 : 0); }


int av1r_flow_debug(uint32_t* pairs, int n, int reset, int* cross_stream)
{
#ifdef AV1R_FLOW_DEBUG
    std::vector<uint32_t> pr(256);
    const int cnt = (int)flow_debug_overlaps(pr.data(), 256, reset);
    int cross = 0;
    std::lock_guard<std::mutex> lock(g_epochMu);
    auto streamOf = [&](uint32_t slot, uint32_t entering) {  // latest epoch < entering in that slot
        hipStream_t s = nullptr, es = nullptr;
        for (auto& e : g_epochLog) {
            if ((e.first & 0xffff) == (entering & 0xffff)) es = e.second;
            if ((e.first & 63) == slot && (e.first & 0xffff) != (entering & 0xffff)) s = e.second;
        }
        return std::make_pair(s, es);
    };
    for (int i = 0; i < std::min(cnt, 256); i++) {
        auto se = streamOf(pr[i] >> 16, pr[i] & 0xffff);
        cross += se.first != se.second;
    }
    if (pairs)
        for (int i = 0; i < n && i < 256; i++) pairs[i] = pr[i];
    if (cross_stream) *cross_stream = cross;
    if (reset) g_epochLog.clear();
    return cnt;
#else
    (void)pairs;
    (void)n;
    (void)reset;
    (void)cross_stream;
    return -1;
#endif
}

int av1r_set_timing(av1r_ctx* c, int enable)
{
    if (!c) return AV1R_E_INVALID;
    c->timing = enable != 0;
    return AV1R_OK;
}

int av1r_set_keep_stages(av1r_ctx* c, int keep)
{
    if (!c) return AV1R_E_INVALID;
    c->keepStages = keep != 0;
    return AV1R_OK;
}

int av1r_last_frame_times(av1r_ctx* c, float* recon, float* lf, float* cdef, float* lr)
{
    if (!c || !c->timing || !c->evUsed) return AV1R_E_INVALID;
    HIPCHK(hipEventSynchronize(c->ev[4]));
    float t[4] = {};
    for (int i = 0; i < 4; i++) HIPCHK(hipEventElapsedTime(&t[i], c->ev[i], c->ev[i + 1]));
    if (recon) *recon = t[0];
    if (lf) *lf = t[1];
    if (cdef) *cdef = t[2];
    if (lr) *lr = t[3];
    return AV1R_OK;
}

int av1r_stage_times(av1r_ctx* c, float* totals, int* frames)
{
    if (!c || !totals) return AV1R_E_INVALID;
    ctx_join(c);
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < 4; i++) totals[i] = 0.f;
    for (size_t f = 0; f < c->evUsed; f++)
        for (int i = 0; i < 4; i++) {
            float t = 0.f;
            HIPCHK(hipEventElapsedTime(&t, c->evPool[f][i], c->evPool[f][i + 1]));
            totals[i] += t;
        }
    if (frames) {
        int nf = 0;
        for (size_t f = 0; f < c->evUsed; f++) nf += c->evFrames[f];
        *frames = nf;
    }
    c->evUsed = 0;
    return AV1R_OK;
}

int av1r_set_schedule(av1r_ctx* c, int mode)
{
    if (!c || mode < -1 || mode > 1) return AV1R_E_INVALID;
    c->schedule = mode;
    return AV1R_OK;
}

int av1r_recon_kernel_times(av1r_ctx* c, float* totals, int* frames)
{
    if (!c || !totals) return AV1R_E_INVALID;
    ctx_join(c);
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < 3; i++) totals[i] = 0.f;
    for (size_t f = 0; f < c->evUsed; f++) {
        const auto& e = c->evPool[f];
        const hipEvent_t seq[4] = {e[0], e[5], e[6], e[1]};  // k_inter, k_resid, k_flow
        for (int i = 0; i < 3; i++) {
            float t = 0.f;
            HIPCHK(hipEventElapsedTime(&t, seq[i], seq[i + 1]));
            totals[i] += t;
        }
    }
    if (frames) {
        int nf = 0;
        for (size_t f = 0; f < c->evUsed; f++) nf += c->evFrames[f];
        *frames = nf;
    }
    return AV1R_OK;
}

int av1r_last_frame_stats(av1r_ctx* c, int* levels, uint64_t* uploadBytes)
{
    if (!c) return AV1R_E_INVALID;
    if (levels) *levels = c->nLevelsLast;
    if (uploadBytes) *uploadBytes = c->lastUploadBytes;
    return AV1R_OK;
}

const char* av1r_last_error(av1r_ctx* c) { return c ? c->err.c_str() : "null context"; }

// Host-only validation + scheduling of a batch (no device): returns the status and, on
// success, the number of dependency levels.  Used by the CPU test-suite.
int av1r_check_batch(const av1r_frame_batch* b, int* levels, char* err, int errLen)
{
    if (!b || !b->hdr) return AV1R_E_INVALID;
    av1r_ctx c;
    c.skipSlotCheck = true;
    int rc = b->hdr->show_existing_frame ? AV1R_OK : validate(&c, b);
    if (!rc && !b->hdr->show_existing_frame) build_schedule(&c, b);
    if (levels) *levels = rc ? 0 : c.nLevelsLast;
    if (err && errLen > 0) snprintf(err, errLen, "%s", c.err.c_str());
    return rc;
}

size_t av1r_sizeof(int which)
{
    switch (which) {
    case 0: return sizeof(av1r_frame_hdr);
    case 1: return sizeof(av1r_mi);
    case 2: return sizeof(av1r_block);
    case 3: return sizeof(av1r_tb);
    case 4: return sizeof(av1r_lr_unit);
    case 5: return sizeof(av1r_frame_batch);
    default: return 0;
    }
}

}  // extern "C"

// ------------------------------------------------------------------------------------
// av1r_ring_sink: pinned host buffers for a pipeline's frame delivery (include/av1r.h)
// ------------------------------------------------------------------------------------
namespace {
struct RingSink {
    int n = 0, w = 0, h = 0, slots = 0;
    size_t frameBytes = 0;
    uint8_t* host = nullptr;  // n * slots frames
    std::vector<int64_t> acquired, delivered;
    std::vector<int> fw, fh;  // per (stream, slot): the frame's size
};

int ring_acquire(void* user, int s, int width, int height, uint8_t** planes, int* strides)
{
    RingSink* R = (RingSink*)user;
    if (!R || s < 0 || s >= R->n || width <= 0 || height <= 0 || width > R->w || height > R->h) return AV1R_E_INVALID;
    if (R->acquired[s] - R->delivered[s] >= R->slots) return AV1R_E_INVALID;  // every buffer is in flight
    const int k = (int)(R->acquired[s]++ % R->slots);
    uint8_t* f = R->host + ((size_t)s * R->slots + k) * R->frameBytes;
    // the library's own frame layout: each read-back is one linear transfer
    const FrameGeom g = frame_geom(width, height);
    for (int p = 0; p < 3; p++) {
        planes[p] = f + g.off[p];
        strides[p] = g.stride[p];
    }
    R->fw[(size_t)s * R->slots + k] = width;
    R->fh[(size_t)s * R->slots + k] = height;
    return AV1R_OK;
}

void ring_deliver(void* user, int s, int status)
{
    RingSink* R = (RingSink*)user;
    if (R && s >= 0 && s < R->n && status == AV1R_OK) R->delivered[s]++;
}
}  // namespace

int av1r_frame_layout(int width, int height, int* strides, size_t* offsets, size_t* span)
{
    if (width <= 0 || height <= 0 || width > 16384 || height > 16384) return AV1R_E_INVALID;
    const FrameGeom g = frame_geom(width, height);
    for (int p = 0; p < 3; p++) {
        if (strides) strides[p] = g.stride[p];
        if (offsets) offsets[p] = g.off[p];
    }
    if (span) *span = g.span;
    return AV1R_OK;
}

int av1r_ring_sink_create(int n_streams, int width, int height, int slots, av1r_output_sink* out)
{
    if (!out || n_streams <= 0 || n_streams > 1024 || width <= 0 || height <= 0 || width > 16384 || height > 16384 ||
        slots < AV1R_SINK_INFLIGHT || slots > 1024)
        return AV1R_E_INVALID;
    RingSink* R = new (std::nothrow) RingSink;
    if (!R) return AV1R_E_NOMEM;
    R->n = n_streams, R->w = width, R->h = height, R->slots = slots;
    R->frameBytes = align256(frame_geom(width, height).span);  // (the largest frame's layout)
    R->acquired.assign(n_streams, 0);
    R->delivered.assign(n_streams, 0);
    R->fw.assign((size_t)n_streams * slots, 0);
    R->fh.assign((size_t)n_streams * slots, 0);
    if (hipHostMalloc((void**)&R->host, R->frameBytes * n_streams * slots, 0) != hipSuccess) {
        delete R;
        return AV1R_E_NOMEM;
    }
    out->acquire = ring_acquire;
    out->deliver = ring_deliver;
    out->user = R;
    return AV1R_OK;
}

void av1r_ring_sink_destroy(av1r_output_sink* sink)
{
    if (!sink || sink->acquire != ring_acquire || !sink->user) return;
    RingSink* R = (RingSink*)sink->user;
    (void)hipHostFree(R->host);
    delete R;
    sink->user = nullptr;
}

int64_t av1r_ring_sink_delivered(const av1r_output_sink* sink, int stream)
{
    if (!sink || sink->acquire != ring_acquire || !sink->user) return -1;
    const RingSink* R = (const RingSink*)sink->user;
    return stream >= 0 && stream < R->n ? R->delivered[stream] : -1;
}

const uint8_t* av1r_ring_sink_frame(const av1r_output_sink* sink, int stream, int64_t k, int* width, int* height)
{
    if (!sink || sink->acquire != ring_acquire || !sink->user) return nullptr;
    const RingSink* R = (const RingSink*)sink->user;
    if (stream < 0 || stream >= R->n || k < 0 || k >= R->delivered[stream] || k < R->acquired[stream] - R->slots) return nullptr;
    const size_t i = (size_t)stream * R->slots + (size_t)(k % R->slots);
    if (width) *width = R->fw[i];
    if (height) *height = R->fh[i];
    return R->host + i * R->frameBytes;
}
