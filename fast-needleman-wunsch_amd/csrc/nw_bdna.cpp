// nw_bdna.cpp -- host helpers of libnwhip.so: .bdna I/O and the seeded
// synthetic-sequence generator (declared in include/nw_hip.h).
#include <cstdio>
#include <cstdlib>

#include "nw_hip.h"

extern "C" {

// readSequence semantics (src/common/helper.cpp:3-25): the whole file, byte by
// byte, no newline stripping; an unopenable file is an error (the reference
// throws std::string(fileName), helper.cpp:5).
int nw_read_bdna(const char *path, int8_t **out, int64_t *n) {
    if (!path || !out || !n) return NW_ERR_ARG;
    *out = nullptr;
    *n = 0;
    FILE *f = std::fopen(path, "rb");
    if (!f) return NW_ERR_ARG;
    int64_t cap = 1 << 16, len = 0;
    int8_t *buf = (int8_t *)std::malloc((size_t)cap);
    if (!buf) {
        std::fclose(f);
        return NW_ERR_OOM;
    }
    for (;;) {
        if (len == cap) {
            cap *= 2;
            int8_t *nb = (int8_t *)std::realloc(buf, (size_t)cap);
            if (!nb) {
                std::free(buf);
                std::fclose(f);
                return NW_ERR_OOM;
            }
            buf = nb;
        }
        size_t got = std::fread(buf + len, 1, (size_t)(cap - len), f);
        len += (int64_t)got;
        if (got == 0) break;
    }
    std::fclose(f);
    *out = buf;
    *n = len;
    return NW_OK;
}

void nw_free(void *p) { std::free(p); }

// i.i.d. uniform bytes in {1,2,3,4} (the .bdna alphabet, README.md:8) from a
// SplitMix64 stream; SURVEY.md 8(d) fixes seeds 1 (s1) and 2 (s2).
void nw_synth_bdna(uint64_t seed, int64_t n, int8_t *out) {
    uint64_t x = seed;
    for (int64_t i = 0; i < n; ++i) {
        x += 0x9E3779B97F4A7C15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        out[i] = (int8_t)(1 + (z >> 62));
    }
}

}  // extern "C"
