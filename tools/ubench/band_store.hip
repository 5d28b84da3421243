// band_store.hip -- chip-wide HBM store rate of the fill's store-wave pattern:
// each storing wave owns a strip of W = 64*C columns and writes it top to bottom,
// NR = 4/C rows per 16-byte-per-lane store instruction (1 KB per instruction),
// strips skewed by `lag` rows (the wavefront skew), persistent over strips.
// Varies the number of storing waves per CU (workgroups x waves per workgroup).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int C>
__global__ void band_store(char *t, long pitchb, long nrows, int nstrips, int lag, int sleepers) {
    constexpr int NR = 4 / C, Q = 16 * C;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    if (wave < sleepers) return;  // idle waves (occupy a slot like a compute wave would)
    const int wpg = blockDim.x / 64 - sleepers;
    const int wid = blockIdx.x * wpg + (wave - sleepers);
    const int nw = gridDim.x * wpg;
    const int ro = lane / Q, cq = lane % Q;
    typedef unsigned v4 __attribute__((ext_vector_type(4)));
    v4 v = {1u, 2u, 3u, (unsigned)lane};
    for (int s = wid; s < nstrips; s += nw) {
        char *base = t + (long)s * (64 * C * 4) + (long)ro * pitchb + cq * 16;
        long r0 = ((long)s * lag) % nrows;
        r0 -= r0 % 64;
        for (long r = 0; r < nrows; r += NR) {
            long row = r + r0;
            if (row >= nrows) row -= nrows;
            *(v4 *)(base + row * pitchb) = v;
            v.x += 1;
        }
    }
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 65536;  // rows and columns
    const long pitch = (n + 64) / 64 * 64 + 64;
    const long pitchb = pitch * 4;
    char *t;
    if (hipMalloc(&t, (size_t)pitchb * (n + 64)) != hipSuccess) { printf("oom\n"); return 1; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](auto kern, int C, int grid, int wpb, int sleepers, int lag) {
        const int nstrips = (int)(n / (64 * C));
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * wpb), 0, 0, t, pitchb, n, nstrips, lag, sleepers);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
        }
        const double bytes = (double)nstrips * 64 * C * 4 * n;
        printf("C=%d grid=%4d waves/WG=%d (idle %d) storing waves=%5d lag=%4d  ms=%7.3f  GB/s=%7.1f\n", C, grid,
               wpb, sleepers, grid * (wpb - sleepers), lag, ms, bytes / (ms * 1e6));
    };
    for (int lag : {128, 512}) {
        run(band_store<2>, 2, 512, 2, 1, lag);   // the fill today: 2 WGs/CU, A idle + B
        run(band_store<2>, 2, 512, 3, 1, lag);   // A + 2 B per WG
        run(band_store<2>, 2, 512, 1, 0, lag);
        run(band_store<2>, 2, 1024, 1, 0, lag);
        run(band_store<2>, 2, 1024, 2, 1, lag);
        run(band_store<4>, 4, 512, 2, 1, lag);
        run(band_store<4>, 4, 512, 3, 1, lag);
        run(band_store<1>, 1, 1024, 2, 1, lag);
    }
    return 0;
}
