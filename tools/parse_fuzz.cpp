// parse_fuzz.cpp -- host-only driver for sanitizer runs of the parser (ASan/UBSan):
// parses every IVF named on the command line, then damaged copies of each temporal unit
// (truncations and bit flips), checking that every outcome is a status, never a fault.
//   g++ -std=c++17 -g -O1 -fsanitize=address,undefined -Iinclude -Iav1dec_amd/csrc/parse \
//       tools/parse_fuzz.cpp av1dec_amd/csrc/parse/{obu,block,api}.cpp -o /tmp/parse_fuzz
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "av1p.h"

static std::vector<std::vector<uint8_t>> ivf_tus(const char* path)
{
    std::vector<std::vector<uint8_t>> out;
    FILE* f = fopen(path, "rb");
    if (!f) return out;
    std::vector<uint8_t> d;
    uint8_t buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof(buf), f)) > 0) d.insert(d.end(), buf, buf + n);
    fclose(f);
    size_t pos = 32;
    while (pos + 12 <= d.size()) {
        const uint32_t sz = d[pos] | d[pos + 1] << 8 | d[pos + 2] << 16 | (uint32_t)d[pos + 3] << 24;
        pos += 12;
        if (pos + sz > d.size()) break;
        out.emplace_back(d.begin() + pos, d.begin() + pos + sz);
        pos += sz;
    }
    return out;
}

int main(int argc, char** argv)
{
    std::mt19937 rng(1234);
    long frames = 0, errors = 0;
    for (int a = 1; a < argc; a++) {
        auto tus = ivf_tus(argv[a]);
        av1p_ctx* c;
        av1p_create(&c);
        for (auto& tu : tus) {
            int n = 0;
            if (av1p_decode_tu(c, tu.data(), tu.size(), &n)) {
                fprintf(stderr, "%s: %s\n", argv[a], av1p_last_error(c));
                return 1;
            }
            frames += n;
        }
        av1p_destroy(c);
        // damaged copies: fresh context per stream, each TU truncated / bit-flipped
        for (int trial = 0; trial < 4; trial++) {
            av1p_create(&c);
            for (auto tu : tus) {
                if (tu.empty()) continue;
                if (trial & 1) tu.resize(rng() % tu.size());
                else
                    for (int k = 0; k < 8; k++) tu[rng() % tu.size()] ^= (uint8_t)(1u << (rng() % 8));
                int n = 0;
                if (av1p_decode_tu(c, tu.data(), tu.size(), &n)) errors++;
            }
            av1p_destroy(c);
        }
    }
    printf("%ld frames parsed, %ld damaged units rejected\n", frames, errors);
    return 0;
}
