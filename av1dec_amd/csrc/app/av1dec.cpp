// av1dec.cpp -- command-line decoder, the counterpart of the reference's test application
// (oddstone/av1dec tests/Av1Dec.cpp): same usage and output formats, built on the drop-in
// YamiAv1::Decoder (include/YamiAv1/Av1Decoder.h).
//
//   av1dec -i input.ivf [-md5] [output.yuv] [-d device]
//
// Reads the IVF container (tests/DecodeInput.cpp: 32-byte file header, 12-byte frame
// headers), decodes every temporal unit, writes the visible I420 planes of each shown frame
// (tests/DecodeOutput.cpp:48-69) and, with -md5, prints "md5=<hex>" of all of them at exit
// (DecodeOutputMd5).  A timing summary like the reference's Fps class goes to stderr.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "YamiAv1/Av1Decoder.h"

namespace {

// MD5 (RFC 1321)
class Md5 {
public:
    Md5() { reset(); }
    void reset()
    {
        h_[0] = 0x67452301;
        h_[1] = 0xefcdab89;
        h_[2] = 0x98badcfe;
        h_[3] = 0x10325476;
        len_ = 0;
        n_ = 0;
    }
    void update(const uint8_t* p, size_t n)
    {
        len_ += n;
        while (n) {
            const size_t k = std::min(n, (size_t)64 - n_);
            memcpy(buf_ + n_, p, k);
            n_ += k;
            p += k;
            n -= k;
            if (n_ == 64) {
                block(buf_);
                n_ = 0;
            }
        }
    }
    std::string hex()
    {
        const uint64_t bits = len_ * 8;
        const uint8_t pad = 0x80;
        update(&pad, 1);
        const uint8_t zero = 0;
        while (n_ != 56) update(&zero, 1);
        uint8_t lenle[8];
        for (int i = 0; i < 8; i++) lenle[i] = (uint8_t)(bits >> (8 * i));
        update(lenle, 8);
        static const char* digits = "0123456789abcdef";
        std::string s;
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) {
                const uint8_t b = (uint8_t)(h_[i] >> (8 * j));
                s += digits[b >> 4];
                s += digits[b & 15];
            }
        return s;
    }

private:
    static uint32_t rol(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }
    void block(const uint8_t* p)
    {
        static const uint32_t K[64] = {
            0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
            0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
            0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
            0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
            0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
            0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
            0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
            0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
        static const int R[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
        uint32_t m[16];
        for (int i = 0; i < 16; i++) m[i] = p[4 * i] | p[4 * i + 1] << 8 | p[4 * i + 2] << 16 | (uint32_t)p[4 * i + 3] << 24;
        uint32_t a = h_[0], b = h_[1], c = h_[2], d = h_[3];
        for (int i = 0; i < 64; i++) {
            uint32_t f;
            int g;
            const int round = i >> 4;
            if (round == 0) f = (b & c) | (~b & d), g = i;
            else if (round == 1) f = (d & b) | (~d & c), g = (5 * i + 1) & 15;
            else if (round == 2) f = b ^ c ^ d, g = (3 * i + 5) & 15;
            else f = c ^ (b | ~d), g = (7 * i) & 15;
            const uint32_t t = d;
            d = c;
            c = b;
            b = b + rol(a + f + K[i] + m[g], R[round * 4 + (i & 3)]);
            a = t;
        }
        h_[0] += a;
        h_[1] += b;
        h_[2] += c;
        h_[3] += d;
    }
    uint32_t h_[4];
    uint64_t len_;
    uint8_t buf_[64];
    size_t n_;
};

void usage(const char* app) { fprintf(stderr, "usage: %s -i input [-md5] [-d device] [output]\n", app); }

}  // namespace

int main(int argc, char** argv)
{
    const char* in = nullptr;
    const char* out = nullptr;
    bool md5 = false;
    int device = 0;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-i") && i + 1 < argc) in = argv[++i];
        else if (!strcmp(argv[i], "-md5")) md5 = true;
        else if (!strcmp(argv[i], "-d") && i + 1 < argc) device = atoi(argv[++i]);
        else if (argv[i][0] != '-' && !out) out = argv[i];
        else {
            usage(argv[0]);
            return -1;
        }
    }
    if (!in) {
        usage(argv[0]);
        return -1;
    }
    FILE* fi = fopen(in, "rb");
    if (!fi) {
        fprintf(stderr, "can't open %s\n", in);
        return -1;
    }
    FILE* fo = nullptr;
    if (out && !(fo = fopen(out, "wb"))) {
        fprintf(stderr, "can't open %s for write\n", out);
        return -1;
    }
    uint8_t hdr[32];
    if (fread(hdr, 1, 32, fi) != 32 || memcmp(hdr, "DKIF", 4)) {
        fprintf(stderr, "fail to read ivf header, quit\n");
        return -1;
    }
    YamiAv1::Decoder decoder(device);
    Md5 sum;
    std::vector<uint8_t> buf;
    long frames = 0, units = 0;
    int status = 0;
    double tDecode = 0, tOut = 0;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto emit = [&]() {
        const auto a = clk::now();
        while (auto f = decoder.getOutput()) {
            for (int p = 0; p < 3; p++)
                for (int y = 0; y < f->heights[p]; y++) {
                    const uint8_t* line = f->data[p] + (size_t)y * f->strides[p];
                    if (fo && fwrite(line, 1, f->widths[p], fo) != (size_t)f->widths[p]) {
                        fprintf(stderr, "write file failed\n");
                        status = -1;
                    }
                    if (md5) sum.update(line, f->widths[p]);
                }
            frames++;
        }
        tOut += std::chrono::duration<double>(clk::now() - a).count();
    };
    uint8_t fh[12];
    while (fread(fh, 1, 12, fi) == 12) {
        const uint32_t sz = fh[0] | fh[1] << 8 | fh[2] << 16 | (uint32_t)fh[3] << 24;
        buf.resize(sz);
        if (fread(buf.data(), 1, sz, fi) != sz) break;
        const auto a = clk::now();
        if (!decoder.decode(buf.data(), buf.size())) {
            fprintf(stderr, "decode failed: %s\n", decoder.lastError().c_str());
            status = -1;
        }
        tDecode += std::chrono::duration<double>(clk::now() - a).count();
        units++;
        emit();
        if (status) break;
    }
    emit();
    const double total = std::chrono::duration<double>(clk::now() - t0).count();
    fprintf(stderr, "%ld units, %ld frames in %.3f s (%.1f fps); decode %.3f s, output %.3f s\n", units, frames, total,
            total > 0 ? frames / total : 0.0, tDecode, tOut);
    if (md5) printf("md5=%s", sum.hex().c_str());
    if (fo) fclose(fo);
    fclose(fi);
    return status;
}
