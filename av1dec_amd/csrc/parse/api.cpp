// api.cpp -- C-ABI of the host parser (include/av1p.h).
#include <algorithm>
#include "parser.h"

#include <stdlib.h>

#include <new>
#include <thread>

#include "av1p.h"

struct av1p_ctx {
    av1p::Parser parser;
    std::vector<av1p::Frame*> frames;
    std::vector<av1p::Frame*> prev;  // av1p_set_frame_generations(ctx, 2): the unit before
    int generations = 1;
    std::string err;
    void recycle(std::vector<av1p::Frame*>& v)
    {
        for (auto* f : v) {
            if (parser.spare.size() < 4) parser.spare.push_back(f);  // (Parser::take_frame)
            else delete f;
        }
        v.clear();
    }
    void release()
    {
        if (generations == 2) {
            recycle(prev);
            prev.swap(frames);
        } else {
            recycle(frames);
        }
    }
    ~av1p_ctx()
    {
        recycle(prev);
        recycle(frames);
    }
};

extern "C" {

int av1p_create(av1p_ctx** out)
{
    if (!out) return AV1R_E_INVALID;
    *out = new (std::nothrow) av1p_ctx;
    if (!*out) return AV1R_E_NOMEM;
    // tile-parallel parsing by default (AV1P_TILE_THREADS overrides; 1 = serial)
    int n = (int)std::thread::hardware_concurrency();
    n = n < 1 ? 1 : n > 8 ? 8 : n;
    if (const char* e = getenv("AV1P_TILE_THREADS")) n = std::min(64, std::max(1, atoi(e)));  // as av1p_set_tile_threads
    (*out)->parser.tile_threads = n;
    return AV1R_OK;
}

int av1p_set_tile_threads(av1p_ctx* ctx, int n)
{
    if (!ctx || n < 1 || n > 64) return AV1R_E_INVALID;
    ctx->parser.tile_threads = n;
    return AV1R_OK;
}

int av1p_set_frame_generations(av1p_ctx* ctx, int n)
{
    if (!ctx || n < 1 || n > 2) return AV1R_E_INVALID;
    ctx->generations = n;
    if (n == 1) ctx->recycle(ctx->prev);
    return AV1R_OK;
}

int av1p_set_mode_info(av1p_ctx* ctx, int emit)
{
    if (!ctx) return AV1R_E_INVALID;
    ctx->parser.emit_mi = emit != 0;
    return AV1R_OK;
}

void av1p_destroy(av1p_ctx* ctx)
{
    if (!ctx) return;
    delete ctx->parser.cur;
    ctx->parser.cur = nullptr;
    for (auto* f : ctx->parser.done) delete f;
    ctx->parser.done.clear();
    delete ctx;
}

int av1p_decode_tu(av1p_ctx* ctx, const uint8_t* data, size_t size, int* n_frames)
{
    if (!ctx || (!data && size)) return AV1R_E_INVALID;
    ctx->release();
    ctx->parser.err.clear();
    int rc;
    try {
        rc = ctx->parser.decode_tu(data, size);
    } catch (const std::bad_alloc&) {
        ctx->parser.err = "out of memory";
        rc = AV1R_E_NOMEM;
    }
    ctx->frames.swap(ctx->parser.done);
    if (rc) {
        // a frame whose tile data failed is not handed out
        delete ctx->parser.cur;
        ctx->parser.cur = nullptr;
        ctx->parser.seen_frame_header = false;
    }
    if (n_frames) *n_frames = (int)ctx->frames.size();
    return rc;
}

const av1r_frame_batch* av1p_frame(av1p_ctx* ctx, int i)
{
    if (!ctx || i < 0 || i >= (int)ctx->frames.size()) return nullptr;
    return &ctx->frames[i]->batch;
}

const char* av1p_last_error(av1p_ctx* ctx) { return ctx ? ctx->parser.err.c_str() : "null context"; }

}  // extern "C"
