// decoder.cpp -- the whole decoder behind the reference's API: YamiAv1::Decoder
// (include/YamiAv1/Av1Decoder.h) and its C-ABI (include/av1dec.h).
//
// Decoder::decode (oddstone/av1dec decoder/Av1Decoder.cpp:49-109) parses a temporal unit and,
// per frame, walks the tile trees (decodeFrame, 128-156) or shows a stored frame
// (showExistingFrame, 158-169).  Here the parse is the host parser (av1p_decode_tu) and each
// parsed frame goes to the MI355X backend as one batch (av1r_decode_frame) -- asynchronous:
// the host parses frame t+1 while the GPU reconstructs frame t.  Every shown frame's read-back
// starts as soon as it is launched (av1r_set_output_prefetch), and getOutput waits for the
// oldest one's copy only (av1r_get_output).
#include <stdlib.h>
#include <string.h>

#include <new>
#include <string>
#include <vector>

#include "YamiAv1/Av1Decoder.h"
#include "av1dec.h"
#include "av1p.h"
#include "av1r.h"

struct av1d_ctx {
    av1p_ctx* parser = nullptr;
    av1r_ctx* recon = nullptr;
    std::string err;
    int fail(int rc, const char* what, const char* detail)
    {
        err = std::string(what) + ": " + (detail ? detail : "");
        return rc;
    }
};

extern "C" {

int av1d_create(int device, av1d_ctx** out)
{
    if (!out) return AV1R_E_INVALID;
    *out = nullptr;
    av1d_ctx* c = new (std::nothrow) av1d_ctx;
    if (!c) return AV1R_E_NOMEM;
    int rc = av1p_create(&c->parser);
    if (!rc) av1p_set_mode_info(c->parser, 0);  // av1r_decode_frame rebuilds it on the device
    if (!rc) rc = av1r_create(device, &c->recon);
    if (rc) {
        av1d_destroy(c);
        return rc;
    }
    av1r_set_keep_stages(c->recon, 0);  // no per-stage snapshots: output only
    // every shown frame's read-back starts as soon as it is decoded, overlapping the parse
    // and decode of the next units; getOutput then waits for that copy alone
    av1r_set_output_prefetch(c->recon, 1);
    *out = c;
    return AV1R_OK;
}

void av1d_destroy(av1d_ctx* c)
{
    if (!c) return;
    if (c->recon) av1r_destroy(c->recon);
    if (c->parser) av1p_destroy(c->parser);
    delete c;
}

int av1d_decode(av1d_ctx* c, const uint8_t* data, size_t size)
{
    if (!c) return AV1R_E_INVALID;
    if (!data || !size) return AV1R_OK;  // end of stream: nothing buffered to flush
    int n = 0;
    int rc = av1p_decode_tu(c->parser, data, size, &n);
    // frames the unit completed before a failure are still reconstructed, as the reference
    // decodes each frame as soon as its last tile group is parsed
    for (int i = 0; i < n; i++) {
        const av1r_frame_batch* b = av1p_frame(c->parser, i);
        const av1r_frame_hdr* h = b->hdr;
        int r = h->show_existing_frame ? av1r_show_existing(c->recon, h->frame_to_show, h->refresh_frame_flags)
                                       : av1r_decode_frame(c->recon, b);
        if (r) return c->fail(r, "reconstruction", av1r_last_error(c->recon));
    }
    if (rc) return c->fail(rc, "parse", av1p_last_error(c->parser));
    return AV1R_OK;
}

int av1d_output_size(av1d_ctx* c, int* width, int* height)
{
    if (!c) return AV1R_E_INVALID;
    if (!av1r_output_pending(c->recon)) return AV1R_E_NO_OUTPUT;
    return av1r_get_output(c->recon, nullptr, 0, nullptr, 0, nullptr, 0, width, height);
}

int av1d_get_output(av1d_ctx* c, uint8_t* y, int ys, uint8_t* u, int us, uint8_t* v, int vs, int* width, int* height)
{
    if (!c) return AV1R_E_INVALID;
    if (!av1r_output_pending(c->recon)) return AV1R_E_NO_OUTPUT;
    const int rc = av1r_get_output(c->recon, y, ys, u, us, v, vs, width, height);
    if (rc) return c->fail(rc, "output", av1r_last_error(c->recon));
    return AV1R_OK;
}

int av1d_flush(av1d_ctx* c)
{
    if (!c) return AV1R_E_INVALID;
    std::vector<uint8_t> scratch;
    int w = 0, h = 0, rc = AV1R_OK;
    while (av1d_output_size(c, &w, &h) == AV1R_OK) {
        const int cw = (w + 1) >> 1, ch = (h + 1) >> 1;
        scratch.resize((size_t)w * h + 2 * (size_t)cw * ch);
        uint8_t* y = scratch.data();
        uint8_t* u = y + (size_t)w * h;
        if ((rc = av1d_get_output(c, y, w, u, cw, u + (size_t)cw * ch, cw, &w, &h))) break;
    }
    return rc;
}

const char* av1d_last_error(av1d_ctx* c) { return c ? c->err.c_str() : "null context"; }

}  // extern "C"

// ---- C++ facade ----
namespace Yami {

// VideoFrame.cpp:41-65: rows padded to 128 + 2 x 16 luma pixels, 16 (luma) / 8 (chroma)
// pixels of margin around every plane, so extendBorder() stays inside the allocation
std::shared_ptr<YuvFrame> YuvFrame::create(int width, int height)
{
    if (width <= 0 || height <= 0) return nullptr;
    std::shared_ptr<YuvFrame> f(new (std::nothrow) YuvFrame);
    if (!f) return nullptr;
    const int pad = 16;
    const size_t aw = (size_t)((width + 127) & ~127) + 2 * pad, ah = (size_t)((height + 127) & ~127) + 2 * pad;
    try {
        f->m_storage.resize(aw * ah * 3 / 2);
    } catch (const std::bad_alloc&) {
        return nullptr;
    }
    f->width = width;
    f->height = height;
    size_t base = 0;
    for (int p = 0; p < MAX_PLANES; p++) {
        const int sub = p ? 2 : 1;
        f->widths[p] = width / sub;
        f->heights[p] = height / sub;
        f->strides[p] = (int)(aw / sub);
        f->data[p] = f->m_storage.data() + base + (size_t)(pad / sub) * f->strides[p] + pad / sub;
        base += (aw / sub) * (ah / sub);
    }
    return f;
}

std::shared_ptr<YuvFrame> YuvFrame::create(const std::shared_ptr<YuvFrame>& other)
{
    if (!other) return nullptr;
    std::shared_ptr<YuvFrame> f = create(other->width, other->height);
    if (!f) return nullptr;
    f->pts = other->pts;
    for (int p = 0; p < MAX_PLANES; p++)
        for (int y = 0; y < other->heights[p]; y++)
            memcpy(f->data[p] + (size_t)y * f->strides[p], other->data[p] + (size_t)y * other->strides[p], other->widths[p]);
    return f;
}

void YuvFrame::extendBorder(int borders)
{
    if (borders <= 0 || borders >= 8) return;  // the margin is 8 chroma pixels
    for (int p = 0; p < MAX_PLANES; p++) {
        const int w = widths[p], h = heights[p], s = strides[p];
        for (int y = 0; y < h; y++) {
            uint8_t* row = data[p] + (size_t)y * s;
            memset(row - borders, row[0], borders);
            memset(row + w, row[w - 1], borders);
        }
        const uint8_t* top = data[p] - borders;
        const uint8_t* bottom = top + (size_t)(h - 1) * s;
        for (int i = 1; i <= borders; i++) {
            memcpy(data[p] - borders - (size_t)i * s, top, w + 2 * borders);
            memcpy(data[p] - borders + (size_t)(h - 1 + i) * s, bottom, w + 2 * borders);
        }
    }
}

}  // namespace Yami

namespace YamiAv1 {

struct Decoder::Impl {
    av1d_ctx* ctx = nullptr;
    int64_t pts = 0;
    std::string err;
};

Decoder::Decoder(int device) : m_impl(new Impl)
{
    const int rc = av1d_create(device, &m_impl->ctx);
    if (rc) m_impl->err = "av1d_create failed with status " + std::to_string(rc);
}

Decoder::~Decoder()
{
    av1d_destroy(m_impl->ctx);
    delete m_impl;
}

bool Decoder::decode(uint8_t* data, size_t size)
{
    if (!m_impl->ctx) return false;
    if (av1d_decode(m_impl->ctx, data, size)) {
        m_impl->err = av1d_last_error(m_impl->ctx);
        return false;
    }
    return true;
}

std::shared_ptr<Yami::YuvFrame> Decoder::getOutput()
{
    if (!m_impl->ctx) return nullptr;
    int w = 0, h = 0;
    if (av1d_output_size(m_impl->ctx, &w, &h)) return nullptr;
    std::shared_ptr<Yami::YuvFrame> f = Yami::YuvFrame::create(w, h);
    if (!f) return nullptr;
    if (av1d_get_output(m_impl->ctx, f->data[0], f->strides[0], f->data[1], f->strides[1], f->data[2], f->strides[2], &w,
                        &h)) {
        m_impl->err = av1d_last_error(m_impl->ctx);
        return nullptr;
    }
    f->pts = m_impl->pts++;
    return f;
}

const std::string& Decoder::lastError() const { return m_impl->err; }

}  // namespace YamiAv1
