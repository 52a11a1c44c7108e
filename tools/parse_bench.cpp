// Host parser timing: parse an IVF file (every temporal unit, in order) `reps` times with
// av1p_decode_tu and print ms per frame.  Links the parser sources directly, so builds with
// other flags (-O3, -march, -pg) can be compared without touching the product build:
//   g++ -std=c++17 -O2 -Iinclude -Iav1dec_amd/csrc/parse tools/parse_bench.cpp
//       av1dec_amd/csrc/parse/{obu,block,api}.cpp -pthread -o /tmp/parse_bench
//   /tmp/parse_bench stream.ivf [reps]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <time.h>

#include "av1p.h"

int main(int argc, char** argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s file.ivf [reps]\n", argv[0]);
        return 2;
    }
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 1;
    std::vector<uint8_t> buf;
    uint8_t tmp[1 << 16];
    size_t n;
    while ((n = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
    fclose(f);
    if (buf.size() < 32 || memcmp(buf.data(), "DKIF", 4) != 0) return 1;
    const size_t hdr = buf[6] | buf[7] << 8;
    std::vector<std::pair<size_t, size_t>> tus;
    for (size_t pos = hdr; pos + 12 <= buf.size();) {
        const size_t sz = buf[pos] | buf[pos + 1] << 8 | buf[pos + 2] << 16 | (size_t)buf[pos + 3] << 24;
        tus.push_back({pos + 12, sz});
        pos += 12 + sz;
    }
    double best = 1e30;
    int frames = 0;
    for (int r = 0; r < reps; r++) {
        av1p_ctx* ctx;
        if (av1p_create(&ctx)) return 1;
        if (getenv("AV1P_NO_MI")) av1p_set_mode_info(ctx, 0);
        frames = 0;
        timespec c0, c1;  // AV1P_CPU_TIME=1: the thread's CPU time (steadier on a shared host)
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c0);
        const auto t0 = std::chrono::steady_clock::now();
        for (auto& tu : tus) {
            int nf = 0;
            if (av1p_decode_tu(ctx, buf.data() + tu.first, tu.second, &nf)) {
                fprintf(stderr, "parse error: %s\n", av1p_last_error(ctx));
                return 1;
            }
            frames += nf;
        }
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c1);
        const double s = getenv("AV1P_CPU_TIME") ? (c1.tv_sec - c0.tv_sec) + 1e-9 * (c1.tv_nsec - c0.tv_nsec)
                                                  : std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        av1p_destroy(ctx);
        if (s < best) best = s;
    }
    printf("%d frames, %.2f ms/frame (best of %d), %.1f KB/frame\n", frames, 1e3 * best / frames, reps,
           (buf.size() - hdr) / 1024.0 / frames);
    return 0;
}
