// yami.cpp -- createVideoDecoder(YAMI_MIME_AV1): the Yami IVideoDecoder the reference declares
// (oddstone/av1dec interface/VideoDecoderHost.h:32-40, VideoDecoderInterface.h:40-66) and never
// implements, over the whole-decoder C-ABI (include/av1dec.h: host parser + MI355X backend).
//
// Status mapping (av1r.h -> VideoCommonDefs.h:130-164): a parse error is
// YAMI_DECODE_PARSER_FAIL, an unsupported stream YAMI_UNSUPPORTED, a device error
// YAMI_DRIVER_FAIL, allocation YAMI_OUT_MEMORY, bad arguments YAMI_INVALID_PARAM; decode()
// before start() is YAMI_NO_CONFIG.
#include <stdlib.h>
#include <string.h>

#include <deque>
#include <new>
#include <vector>

#include "av1dec.h"
#include "av1r.h"
#include "yami/yami_av1.h"

namespace {

using namespace YamiMediaCodec;

YamiStatus to_yami(int rc, bool parse)
{
    switch (rc) {
    case AV1R_OK: return YAMI_SUCCESS;
    case AV1R_E_UNSUPPORTED: return YAMI_UNSUPPORTED;
    case AV1R_E_NOMEM: return YAMI_OUT_MEMORY;
    case AV1R_E_DEVICE: return YAMI_DRIVER_FAIL;
    default: return parse ? YAMI_DECODE_PARSER_FAIL : YAMI_FAIL;
    }
}

// one output frame: the VideoFrame, its raw-data descriptor and the I420 pixels in one block
struct OutFrame {
    VideoFrame frame;
    VideoFrameRawData raw;
    uint8_t pixels[1];
};

void free_out_frame(VideoFrame* f)
{
    if (f) free((void*)f->user_data);
}

class Av1Decoder : public IVideoDecoder {
public:
    ~Av1Decoder() override { stop(); }

    YamiStatus start(VideoConfigBuffer* buffer) override
    {
        stop();
        const char* dev = getenv("AV1R_DEVICE");
        const int rc = av1d_create(dev ? atoi(dev) : 0, &m_ctx);
        if (rc) {
            m_ctx = nullptr;
            return rc == AV1R_E_NOMEM ? YAMI_OUT_MEMORY : YAMI_DRIVER_FAIL;
        }
        m_wantW = buffer ? buffer->width : 0;
        m_wantH = buffer ? buffer->height : 0;
        memset(&m_info, 0, sizeof(m_info));
        m_info.mimeType = m_mime;
        m_info.fourcc = YAMI_FOURCC_I420;
        m_pts.clear();
        return YAMI_SUCCESS;
    }

    YamiStatus reset(VideoConfigBuffer* buffer) override { return start(buffer); }

    void stop() override
    {
        if (m_ctx) av1d_destroy(m_ctx);
        m_ctx = nullptr;
        m_pts.clear();
        m_changed.clear();
    }

    void flush() override
    {
        if (!m_ctx) return;
        av1d_flush(m_ctx);
        m_pts.clear();
        m_changed.clear();
    }

    YamiStatus decode(VideoDecodeBuffer* buffer) override
    {
        if (!m_ctx) return YAMI_NO_CONFIG;
        if (!buffer || !buffer->data || !buffer->size) return YAMI_SUCCESS;  // end of stream
        // A libyami client answers YAMI_DECODE_FORMAT_CHANGE by reconfiguring and sending the
        // same buffer again.  This decoder has already decoded that unit (its frames are
        // queued), so the resend is acknowledged without decoding it twice (which would
        // duplicate its output, refresh the reference slots again and shift the pts queue).
        if (!m_changed.empty()) {
            const bool resend = buffer->size == m_changed.size() && buffer->timeStamp == m_changedTs &&
                                memcmp(buffer->data, m_changed.data(), buffer->size) == 0;
            m_changed.clear();
            if (resend) return YAMI_SUCCESS;
        }
        const int rc = av1d_decode(m_ctx, buffer->data, buffer->size);
        const bool parse = strncmp(av1d_last_error(m_ctx), "parse", 5) == 0;
        if (rc) return to_yami(rc, parse);
        m_pts.push_back(buffer->timeStamp);
        int w, h;
        if (av1d_output_size(m_ctx, &w, &h) == AV1R_OK && ((uint32_t)w != m_info.width || (uint32_t)h != m_info.height)) {
            m_info.valid = true;
            m_info.width = (uint32_t)w;
            m_info.height = (uint32_t)h;
            m_info.surfaceWidth = (uint32_t)((w + 7) & ~7);
            m_info.surfaceHeight = (uint32_t)((h + 7) & ~7);
            m_info.surfaceNumber = 8 + 2;  // the 8 reference slots + output in flight
            m_info.cropRight = w;
            m_info.cropBottom = h;
            if ((m_wantW && m_wantW != (uint32_t)w) || (m_wantH && m_wantH != (uint32_t)h)) {
                m_wantW = (uint32_t)w;
                m_wantH = (uint32_t)h;
                m_changed.assign(buffer->data, buffer->data + buffer->size);
                m_changedTs = buffer->timeStamp;
                return YAMI_DECODE_FORMAT_CHANGE;
            }
        }
        return YAMI_SUCCESS;
    }

    SharedPtr<VideoFrame> getOutput() override
    {
        if (!m_ctx) return nullptr;
        int w = 0, h = 0;
        if (av1d_output_size(m_ctx, &w, &h) != AV1R_OK) return nullptr;
        const int cw = (w + 1) >> 1, ch = (h + 1) >> 1;
        const size_t ySize = (size_t)w * h, cSize = (size_t)cw * ch;
        OutFrame* o = (OutFrame*)malloc(sizeof(OutFrame) + ySize + 2 * cSize);
        if (!o) return nullptr;
        memset(o, 0, sizeof(OutFrame));
        uint8_t* y = o->pixels;
        if (av1d_get_output(m_ctx, y, w, y + ySize, cw, y + ySize + cSize, cw, &w, &h) != AV1R_OK) {
            free(o);
            return nullptr;
        }
        VideoFrameRawData& r = o->raw;
        r.memoryType = VIDEO_DATA_MEMORY_TYPE_RAW_POINTER;
        r.width = (uint32_t)w;
        r.height = (uint32_t)h;
        r.pitch[0] = (uint32_t)w;
        r.pitch[1] = r.pitch[2] = (uint32_t)cw;
        r.offset[0] = 0;
        r.offset[1] = (uint32_t)ySize;
        r.offset[2] = (uint32_t)(ySize + cSize);
        r.fourcc = YAMI_FOURCC_I420;
        r.size = (uint32_t)(ySize + 2 * cSize);
        r.handle = (intptr_t)y;
        VideoFrame& f = o->frame;
        f.surface = (intptr_t)&o->raw;
        if (!m_pts.empty()) {  // shown frames come out in input order (one per unit here)
            f.timeStamp = m_pts.front();
            m_pts.pop_front();
        }
        r.timeStamp = f.timeStamp;
        f.crop.width = (uint32_t)w;
        f.crop.height = (uint32_t)h;
        f.fourcc = YAMI_FOURCC_I420;
        f.user_data = (intptr_t)o;
        f.free = free_out_frame;
        return SharedPtr<VideoFrame>(&o->frame, [](VideoFrame* p) { p->free(p); });
    }

    const VideoFormatInfo* getFormatInfo() override { return m_info.valid ? &m_info : nullptr; }
    void setNativeDisplay(NativeDisplay*) override {}
    void setAllocator(SurfaceAllocator*) override {}
    void releaseLock(bool) override {}

private:
    av1d_ctx* m_ctx = nullptr;
    VideoFormatInfo m_info = {};
    uint32_t m_wantW = 0, m_wantH = 0;
    std::deque<int64_t> m_pts;
    std::vector<uint8_t> m_changed;  // the unit that reported YAMI_DECODE_FORMAT_CHANGE (a resend is a no-op)
    int64_t m_changedTs = 0;
    char m_mime[32] = YAMI_MIME_AV1;
};

}  // namespace

extern "C" {

IVideoDecoder* createVideoDecoder(const char* mimeType)
{
    if (!mimeType || strcmp(mimeType, YAMI_MIME_AV1) != 0) return nullptr;
    return new (std::nothrow) Av1Decoder;
}

void releaseVideoDecoder(IVideoDecoder* p) { delete p; }

}  // extern "C"
