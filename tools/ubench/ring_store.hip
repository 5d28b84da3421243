// ring_store.hip -- HBM store rate of a strip sweep whose CU strip (1 KB per row)
// is written as NRING sub-strips ("rings") of 1024/NRING bytes, ring k lagging
// ring k-1 by LAGR rows (chained compute waves), each ring drained by SPR store
// waves taking B-row batches round robin.  One store instruction covers R rows x
// 1024/R bytes (16 B per lane); a ring row of W bytes takes W*R/1024 of them.
// Strips are claimed persistently (strip s by workgroup s % grid), strip s
// starting at row (s * lag) mod nrows and wrapping.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int NRING, int R>
__global__ void ring_store(char *t, long pitchb, long nrows, int spr, int B, int nstrips, int lag, int lagr) {
    constexpr int W = 1024 / NRING;        // bytes per ring row
    constexpr int PB = 1024 / R;           // bytes per row of one instruction
    constexpr int NP = W / PB;             // instructions per R ring rows
    static_assert(NP >= 1, "shape");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ring = wave % NRING, q = wave / NRING;
    const int ro = lane / (64 / R), cq = lane % (64 / R);
    typedef unsigned v4 __attribute__((ext_vector_type(4)));
    v4 v = {1u, 2u, 3u, (unsigned)lane};
    for (int s = blockIdx.x; s < nstrips; s += gridDim.x) {
        long r0 = ((long)s * lag + (long)ring * lagr) % nrows;
        char *base = t + (long)s * 1024 + ring * W + (long)ro * pitchb + cq * 16;
        for (long f = (long)q * B; f < nrows; f += (long)spr * B) {
            for (int g = 0; g < B; g += R) {
                if (f + g >= nrows) break;
                long row = f + g + r0;
                if (row >= nrows) row -= nrows;
#pragma unroll
                for (int p = 0; p < NP; ++p) *(v4 *)(base + row * pitchb + p * PB) = v;
                v.x += 1;
            }
        }
    }
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 262144;
    const long pitchb = (n + 64) * 4;  // the fill's pitch: n1 + 4 rounded up to 64 columns
    char *t;
    if (hipMalloc(&t, (size_t)pitchb * n) != hipSuccess) { printf("oom\n"); return 1; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](auto kern, const char *name, int nring, int spr, int B, int lagr) {
        const int nstrips = (int)(n * 4 / 1024);
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(256), dim3(64 * nring * spr), 0, 0, t, pitchb, n, spr, B, nstrips, 192, lagr);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
        }
        const double bytes = (double)n * 4 * n;
        printf("%-26s rings=%d store waves/ring=%d B=%2d ring lag=%3d ms=%7.3f GB/s=%7.1f\n", name, nring, spr, B, lagr,
               ms, bytes / (ms * 1e6));
    };
    run(ring_store<2, 2>, "2 rings, 2 rows x 512 B", 2, 2, 16, 80);   // the fill today
    run(ring_store<4, 8>, "4 rings, 8 rows x 128 B", 4, 1, 16, 80);
    run(ring_store<4, 8>, "4 rings, 8 rows x 128 B", 4, 1, 32, 80);
    run(ring_store<4, 8>, "4 rings, 8 rows x 128 B", 4, 2, 16, 80);
    run(ring_store<4, 4>, "4 rings, 4 rows x 256 B", 4, 1, 16, 80);
    run(ring_store<4, 4>, "4 rings, 4 rows x 256 B", 4, 2, 16, 80);
    run(ring_store<4, 8>, "4 rings, 8 rows x 128 B", 4, 1, 16, 0);
    run(ring_store<1, 1>, "1 ring, 1 row x 1 KB", 1, 4, 16, 0);
    run(ring_store<2, 8>, "2 rings, 8 rows x 128 B", 2, 2, 16, 80);
    return 0;
}
