// gprof driver for tools/parse_gprof.sh: parse an IVF file N times with the host parser (no GPU)
#include "av1p.h"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb"); std::vector<uint8_t> d; uint8_t buf[65536]; size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) d.insert(d.end(), buf, buf + n);
    fclose(f);
    int reps = argc > 2 ? atoi(argv[2]) : 3, frames = 0;
    for (int r = 0; r < reps; r++) {
        av1p_ctx* c; av1p_create(&c); av1p_set_mode_info(c, 0); av1p_set_tile_threads(c, 1);
        size_t pos = 32;
        while (pos + 12 <= d.size()) {
            uint32_t sz; memcpy(&sz, &d[pos], 4); pos += 12;
            int nf = 0; if (av1p_decode_tu(c, &d[pos], sz, &nf)) { fprintf(stderr, "err %s\n", av1p_last_error(c)); return 1; }
            frames += nf; pos += sz;
        }
        av1p_destroy(c);
    }
    printf("frames %d\n", frames);
}
