// Av1Decoder.h -- drop-in for the reference decoder's public class (oddstone/av1dec,
// decoder/Av1Decoder.h:47-70; the frame type is VideoFrame.h's): the same names, signatures and
// semantics, backed by the host parser (include/av1p.h) and the MI355X reconstruction
// backend (include/av1r.h).  An application written against YamiAv1::Decoder -- like the
// reference's own tests/Av1Dec.cpp -- rebuilds against this directory and libav1r.so unchanged
// (tests/test_yami.py compiles and links it).
//
//   YamiAv1::Decoder decoder;                    // Decoder::Decoder (Av1Decoder.cpp:40-43)
//   decoder.decode(data, size);                  // one temporal unit (Av1Decoder.cpp:49-109)
//   while (auto f = decoder.getOutput()) ...     // shown frames in order (Av1Decoder.cpp:203-211)
//
// Differences, by design: decode() runs reconstruction and filtering on the GPU
// asynchronously and getOutput() waits for the frame it returns; device errors surface as
// decode() == false or a null getOutput(), with lastError() describing them.
#ifndef YAMIAV1_AV1DECODER_H
#define YAMIAV1_AV1DECODER_H

#include <stddef.h>
#include <stdint.h>

#include <memory>
#include <string>

#include "VideoFrame.h"  // Yami::YuvFrame (decoder/VideoFrame.h:34-58)

namespace YamiAv1 {

class Decoder {
public:
    // device: HIP device ordinal (the reference has no device; 0 by default)
    explicit Decoder(int device = 0);
    ~Decoder();
    Decoder(const Decoder&) = delete;
    Decoder& operator=(const Decoder&) = delete;
    // Parse one temporal unit and queue its frames for reconstruction (returns false on a
    // parse error, an unsupported stream or a device error).
    bool decode(uint8_t* data, size_t size);
    // The oldest shown frame not yet returned, or nullptr if none is pending.
    std::shared_ptr<Yami::YuvFrame> getOutput();
    // Not in the reference: the message of the last failure.
    const std::string& lastError() const;

private:
    struct Impl;
    Impl* m_impl;
};

}  // namespace YamiAv1

#endif
