// yami_av1.h -- the Yami decoder interface the reference declares but never implements,
// implemented for AV1 by libav1r.so (av1dec_amd/csrc/app/yami.cpp).
//
// The reference's interface/ directory (oddstone/av1dec: Yami.h, VideoDecoderHost.h:32-40,
// VideoDecoderInterface.h:40-66, VideoDecoderDefs.h, VideoCommonDefs.h:130-164,257-283) is
// restated here for the decoder side only -- the same type names, member order and enum values,
// so an application built against the reference's headers links against libav1r.so unchanged
// (tests/test_yami.py builds one against each).  Encoder and post-processing declarations
// are left out.
//
// Output frames are software frames in host memory: VideoFrame::surface points to a
// VideoFrameRawData (memoryType VIDEO_DATA_MEMORY_TYPE_RAW_POINTER, fourcc I420, `handle` the
// buffer, `pitch` / `offset` per plane); the SharedPtr returned by getOutput() frees both.
#ifndef YAMI_AV1_H
#define YAMI_AV1_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
#include <memory>
#define SharedPtr std::shared_ptr
#define WeakPtr std::weak_ptr
#define DynamicPointerCast std::dynamic_pointer_cast
#define StaticPointerCast std::static_pointer_cast
#define EnableSharedFromThis std::enable_shared_from_this
extern "C" {
#endif

#define YAMI_FOURCC(a, b, c, d) \
    ((uint32_t)(uint8_t)(a) | ((uint32_t)(uint8_t)(b) << 8) | ((uint32_t)(uint8_t)(c) << 16) | ((uint32_t)(uint8_t)(d) << 24))
#define YAMI_FOURCC_I420 YAMI_FOURCC('I', '4', '2', '0')
#define YAMI_FOURCC_NV12 YAMI_FOURCC('N', 'V', '1', '2')
#define YAMI_FOURCC_YV12 YAMI_FOURCC('Y', 'V', '1', '2')

#define YAMI_MIME_AV1 "video/x-vnd.on2.av1"

// status codes (values of VideoCommonDefs.h:130-164: fatal errors count up from -1024)
typedef enum {
    YAMI_FATAL_ERROR = -1024,
    YAMI_DECODE_PARSER_FAIL,
    YAMI_FAIL,
    YAMI_NO_CONFIG,
    YAMI_DRIVER_FAIL,
    YAMI_NOT_IMPLEMENT,
    YAMI_UNSUPPORTED,
    YAMI_INVALID_PARAM,
    YAMI_OUT_MEMORY,
    YAMI_SUCCESS = 0,
    YAMI_MORE_DATA,
    YAMI_DECODE_INVALID_DATA,
    YAMI_DECODE_FORMAT_CHANGE,
    YAMI_DECODE_NO_SURFACE,
    YAMI_ENCODE_BUFFER_TOO_SMALL,
    YAMI_ENCODE_BUFFER_NO_MORE,
    YAMI_ENCODE_IS_BUSY,
    YAMI_ENCODE_NO_REQUEST_DATA,
} YamiStatus;
typedef YamiStatus Decode_Status;

typedef enum {
    NATIVE_DISPLAY_AUTO,
    NATIVE_DISPLAY_X11,
    NATIVE_DISPLAY_DRM,
    NATIVE_DISPLAY_WAYLAND,
    NATIVE_DISPLAY_VA,
} YamiNativeDisplayType;

typedef struct NativeDisplay {
    intptr_t handle;
    YamiNativeDisplayType type;
} NativeDisplay;

typedef enum {
    VIDEO_DATA_MEMORY_TYPE_RAW_POINTER,
    VIDEO_DATA_MEMORY_TYPE_RAW_COPY,
    VIDEO_DATA_MEMORY_TYPE_DRM_NAME,
    VIDEO_DATA_MEMORY_TYPE_DMA_BUF,
    VIDEO_DATA_MEMORY_TYPE_SURFACE_ID,
    VIDEO_DATA_MEMORY_TYPE_ANDROID_BUFFER_HANDLE,
    VIDEO_DATA_MEMORY_TYPE_EXTERNAL_DMA_BUF,
} VideoDataMemoryType;

typedef struct VideoFrameRawData {
    VideoDataMemoryType memoryType;
    uint32_t width;
    uint32_t height;
    uint32_t pitch[3];
    uint32_t offset[3];
    uint32_t fourcc;
    uint32_t size;
    intptr_t handle;
    uint32_t internalID;
    int64_t timeStamp;
    uint32_t flags;
} VideoFrameRawData;

#define VIDEO_FRAME_FLAGS_KEY 1

typedef struct _SurfaceAllocParams SurfaceAllocParams;
struct _SurfaceAllocParams {
    uint32_t fourcc;
    uint32_t width;
    uint32_t height;
    uint32_t size;
    intptr_t* surfaces;
    YamiStatus (*getSurface)(SurfaceAllocParams* thiz, intptr_t* surface);
    YamiStatus (*putSurface)(SurfaceAllocParams* thiz, intptr_t surface);
    void* user;
};

typedef struct _SurfaceAllocator SurfaceAllocator;
struct _SurfaceAllocator {
    void* user;
    YamiStatus (*alloc)(SurfaceAllocator* thiz, SurfaceAllocParams* params);
    YamiStatus (*free)(SurfaceAllocator* thiz, SurfaceAllocParams* params);
    void (*unref)(SurfaceAllocator* thiz);
};

typedef struct VideoRect {
    uint32_t x;
    uint32_t y;
    uint32_t width;
    uint32_t height;
} VideoRect;

typedef struct VideoFrame {
    intptr_t surface;  // here: a VideoFrameRawData* (see the file comment)
    int64_t timeStamp;
    VideoRect crop;
    uint32_t flags;
    uint32_t fourcc;
    intptr_t user_data;
    void (*free)(struct VideoFrame*);
} VideoFrame;

// decoder buffers (VideoDecoderDefs.h)
typedef enum {
    HAS_SURFACE_NUMBER = 0x04,
    HAS_VA_PROFILE = 0x08,
} VIDEO_BUFFER_FLAG;

typedef struct {
    uint8_t* data;
    size_t size;
    int64_t timeStamp;
    uint32_t flag;
} VideoDecodeBuffer;

typedef struct {
    uint8_t* data;
    int32_t size;
    uint32_t width;
    uint32_t height;
    int32_t surfaceWidth;
    int32_t surfaceHeight;
    int32_t frameRate;
    int32_t surfaceNumber;
    uint32_t flag;
    uint32_t fourcc;
    uint32_t temporalLayer;
    uint32_t spacialLayer;
    uint32_t qualityLayer;
} VideoConfigBuffer;

typedef struct {
    bool valid;
    char* mimeType;
    uint32_t width;
    uint32_t height;
    uint32_t surfaceWidth;
    uint32_t surfaceHeight;
    uint32_t surfaceNumber;
    int32_t aspectX;
    int32_t aspectY;
    int32_t cropLeft;
    int32_t cropRight;
    int32_t cropTop;
    int32_t cropBottom;
    int32_t colorMatrix;
    int32_t videoRange;
    int32_t bitrate;
    int32_t framerateNom;
    int32_t framerateDenom;
    uint32_t fourcc;
} VideoFormatInfo;

#ifdef __cplusplus
}  // extern "C"

namespace YamiMediaCodec {

// VideoDecoderInterface.h:40-66; virtual member order is the ABI
class IVideoDecoder {
public:
    virtual ~IVideoDecoder() {}
    // configure before the first decode; a stream whose size differs from a non-zero
    // buffer->width/height makes decode() return YAMI_DECODE_FORMAT_CHANGE (the unit is decoded)
    virtual YamiStatus start(VideoConfigBuffer* buffer) = 0;
    // stop, then start with `buffer`: pending input and frames are discarded
    virtual YamiStatus reset(VideoConfigBuffer* buffer) = 0;
    virtual void stop(void) = 0;
    // drop frames not yet returned (seek); the next unit should start at a key frame
    virtual void flush(void) = 0;
    // one temporal unit; data NULL / size 0 is end of stream
    virtual YamiStatus decode(VideoDecodeBuffer* buffer) = 0;
    // the next shown frame, or null
    virtual SharedPtr<VideoFrame> getOutput() = 0;
    virtual const VideoFormatInfo* getFormatInfo(void) = 0;
    // hardware-display hooks: accepted and unused (frames are host memory)
    virtual void setNativeDisplay(NativeDisplay* display = NULL) = 0;
    virtual void setAllocator(SurfaceAllocator* allocator) = 0;
    virtual void releaseLock(bool lockable = false) = 0;
};

}  // namespace YamiMediaCodec

// VideoDecoderHost.h:32-40 (extern "C" for dlsym)
extern "C" {
YamiMediaCodec::IVideoDecoder* createVideoDecoder(const char* mimeType);
void releaseVideoDecoder(YamiMediaCodec::IVideoDecoder* p);
typedef YamiMediaCodec::IVideoDecoder* (*YamiCreateVideoDecoderFuncPtr)(const char* mimeType);
typedef void (*YamiReleaseVideoDecoderFuncPtr)(YamiMediaCodec::IVideoDecoder* p);
}
#endif  // __cplusplus

#endif
