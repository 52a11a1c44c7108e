// yami_decode.cpp -- an application of the Yami decoder API (include/yami/yami_av1.h): the
// IVF file in, I420 frames out, through createVideoDecoder(YAMI_MIME_AV1) alone -- the way a
// libyami client (the reference's interface/VideoDecoderHost.h:32-40) drives a decoder.
//
//   yami_decode <in.ivf> <out.yuv> [--size WxH] [--flush-at N]
//
// --size passes the expected dimensions to start() (a stream of another size reports
// YAMI_DECODE_FORMAT_CHANGE once, and the buffer is sent again, as libyami clients do);
// --flush-at N calls flush() after unit N and skips to the
// next key frame (seek).  Exit status 0 on success; the status of a failing call otherwise.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "yami/yami_av1.h"

using namespace YamiMediaCodec;

static bool read_file(const char* path, std::vector<uint8_t>& out)
{
    FILE* f = fopen(path, "rb");
    if (!f) return false;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof(buf), f)) > 0) out.insert(out.end(), buf, buf + n);
    fclose(f);
    return true;
}

static uint32_t le32(const uint8_t* p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }

static bool is_key_unit(const uint8_t* d, size_t n)
{
    // a temporal unit whose first frame header is a shown key frame: scan the OBUs
    size_t pos = 0;
    while (pos < n) {
        const int type = (d[pos] >> 3) & 15;
        const bool ext = d[pos] & 4, hasSize = d[pos] & 2;
        size_t h = 1 + ext, sz = 0;
        if (hasSize) {
            for (int i = 0; i < 8 && pos + h < n; i++) {
                sz |= (size_t)(d[pos + h] & 0x7f) << (7 * i);
                if (!(d[pos + h++] & 0x80)) break;
            }
        } else {
            sz = n - pos - h;
        }
        if ((type == 3 || type == 6) && pos + h < n) {
            const uint8_t b = d[pos + h];  // show_existing_frame(1) frame_type(2) show_frame(1)
            return !(b & 0x80) && ((b >> 5) & 3) == 0 && (b & 0x10);
        }
        pos += h + sz;
    }
    return false;
}

int main(int argc, char** argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s <in.ivf> <out.yuv> [--size WxH] [--flush-at N]\n", argv[0]);
        return 2;
    }
    VideoConfigBuffer cfg;
    memset(&cfg, 0, sizeof(cfg));
    int flushAt = -1;
    for (int i = 3; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "--size")) sscanf(argv[i + 1], "%ux%u", &cfg.width, &cfg.height);
        else if (!strcmp(argv[i], "--flush-at")) flushAt = atoi(argv[i + 1]);
    }
    std::vector<uint8_t> ivf;
    if (!read_file(argv[1], ivf) || ivf.size() < 32 || memcmp(ivf.data(), "DKIF", 4)) {
        fprintf(stderr, "cannot read IVF %s\n", argv[1]);
        return 2;
    }
    FILE* out = fopen(argv[2], "wb");
    if (!out) return 2;
    IVideoDecoder* dec = createVideoDecoder(YAMI_MIME_AV1);
    if (!dec) {
        fprintf(stderr, "createVideoDecoder(%s) returned NULL\n", YAMI_MIME_AV1);
        return 3;
    }
    YamiStatus st = dec->start(&cfg);
    if (st != YAMI_SUCCESS) {
        fprintf(stderr, "start: status %d\n", st);
        releaseVideoDecoder(dec);
        return 4;
    }
    int frames = 0, formatChanges = 0, unit = 0;
    bool skipping = false;
    auto drain = [&]() {
        while (SharedPtr<VideoFrame> f = dec->getOutput()) {
            const VideoFrameRawData* r = (const VideoFrameRawData*)f->surface;
            const uint8_t* base = (const uint8_t*)r->handle;
            for (int p = 0; p < 3; p++) {
                const uint32_t w = p ? (r->width + 1) >> 1 : r->width, h = p ? (r->height + 1) >> 1 : r->height;
                for (uint32_t y = 0; y < h; y++) fwrite(base + r->offset[p] + (size_t)y * r->pitch[p], 1, w, out);
            }
            frames++;
        }
    };
    size_t pos = 32;
    while (pos + 12 <= ivf.size()) {
        const uint32_t sz = le32(&ivf[pos]);
        VideoDecodeBuffer buf;
        memset(&buf, 0, sizeof(buf));
        buf.data = &ivf[pos + 12];
        buf.size = sz;
        buf.timeStamp = unit;
        pos += 12 + sz;
        if (skipping && !is_key_unit(buf.data, buf.size)) {
            unit++;
            continue;
        }
        skipping = false;
        st = dec->decode(&buf);
        if (st == YAMI_DECODE_FORMAT_CHANGE) {
            const VideoFormatInfo* fi = dec->getFormatInfo();
            fprintf(stderr, "format change: %ux%u\n", fi ? fi->width : 0, fi ? fi->height : 0);
            formatChanges++;
            st = dec->decode(&buf);  // as libyami clients do: reconfigure, then send the buffer again
        }
        if (st != YAMI_SUCCESS) {
            fprintf(stderr, "decode unit %d: status %d\n", unit, st);
            releaseVideoDecoder(dec);
            return 5;
        }
        drain();
        if (unit == flushAt) {
            dec->flush();
            skipping = true;
        }
        unit++;
    }
    VideoDecodeBuffer eos;
    memset(&eos, 0, sizeof(eos));
    dec->decode(&eos);
    drain();
    const VideoFormatInfo* fi = dec->getFormatInfo();
    printf("frames=%d format_changes=%d size=%ux%u fourcc_i420=%d\n", frames, formatChanges, fi ? fi->width : 0,
           fi ? fi->height : 0, fi && fi->fourcc == YAMI_FOURCC_I420);
    dec->stop();
    releaseVideoDecoder(dec);
    fclose(out);
    return 0;
}
