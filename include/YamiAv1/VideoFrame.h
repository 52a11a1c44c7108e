// VideoFrame.h -- Yami::YuvFrame, the frame type of the reference's public API
// (oddstone/av1dec decoder/VideoFrame.h:34-58, VideoFrame.cpp:41-101), for applications
// built against include/YamiAv1 and libav1r.so: the same members, with the same meaning.
//
// An 8-bit I420 frame in host memory.  Plane p is widths[p] x heights[p] pixels (chroma:
// half the luma size), rows strides[p] bytes apart; every plane has a 16-pixel margin (8
// for chroma) on each side, inside the allocation, so extendBorder() may replicate up to 7
// pixels outward, as the reference's loop restoration does before reading across the edge.
#ifndef YAMIAV1_VIDEOFRAME_H
#define YAMIAV1_VIDEOFRAME_H

#include <stdint.h>

#include <memory>
#include <vector>

namespace Yami {

struct YuvFrame {
    static const int MAX_PLANES = 3;
    int64_t pts = 0;
    int width = 0;
    int height = 0;
    uint8_t* data[MAX_PLANES] = {};
    int strides[MAX_PLANES] = {};
    int widths[MAX_PLANES] = {};
    int heights[MAX_PLANES] = {};
    // a frame of width x height (contents undefined)
    static std::shared_ptr<YuvFrame> create(int width, int height);
    // a copy of other's pixels (VideoFrame.cpp:67-82)
    static std::shared_ptr<YuvFrame> create(const std::shared_ptr<YuvFrame>& other);
    inline uint8_t getPixel(int plane, int x, int y) const;
    inline void setPixel(int plane, int x, int y, uint8_t pixel);
    // replicate each plane's edge pixels `borders` (< 8) pixels outward (VideoFrame.cpp:84-101)
    void extendBorder(int borders);

private:
    std::vector<uint8_t> m_storage;
};

inline uint8_t YuvFrame::getPixel(int plane, int x, int y) const { return data[plane][y * strides[plane] + x]; }

inline void YuvFrame::setPixel(int plane, int x, int y, uint8_t pixel) { data[plane][y * strides[plane] + x] = pixel; }

}  // namespace Yami

#endif
