// cadence_store.hip -- store bandwidth under the fill's per-wave cadence.
// Persistent single-wave workgroups sweep 64-column strips (like the fill):
// per iteration (64 rows) a wave issues NLOAD dword loads (prefetch), 16 x
// dwordx4 stores (one 64-row x 256-B block), then "computes" for DELAY cycles,
// and consumes the loads issued DIST iterations earlier (an s_waitcnt that, with
// in-order vmcnt, also drains every older store).  Strips are skewed by 64*LAGB
// rows with wrap-around, so every store stays inside the table.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int NLOAD, int DIST>
__global__ __launch_bounds__(64) void cadence(int *t, const int *src, long pitch, long nblocks,
                                              int nstrips, long lagb, int delay, int *sink) {
    const int lane = threadIdx.x;
    const int rsub = lane >> 4, csub = (lane & 15) * 4;
    int acc = 0;
    for (int strip = blockIdx.x; strip < nstrips; strip += gridDim.x) {
        long shift = ((long)strip * lagb) % nblocks;
        int ring[DIST + 1][NLOAD > 0 ? NLOAD : 1];
#pragma unroll
        for (int d = 0; d <= DIST; ++d)
#pragma unroll
            for (int j = 0; j < (NLOAD > 0 ? NLOAD : 1); ++j) ring[d][j] = 0;
        // iterations unrolled by DIST+1 so the prefetch ring is indexed at compile time
        for (long k0 = 0; k0 + DIST + 1 <= nblocks; k0 += DIST + 1) {
#pragma unroll
            for (int ph = 0; ph <= DIST; ++ph) {
                const long k = k0 + ph;
                if constexpr (NLOAD > 0) {
#pragma unroll
                    for (int j = 0; j < NLOAD; ++j)
                        ring[(ph + DIST) % (DIST + 1)][j] = src[((k * 64 + j * 64 + lane) & 0xFFFFF)];
                }
                long blk = k - shift;
                if (blk < 0) blk += nblocks;
                int *base = t + (blk * 64 + rsub) * pitch + (long)strip * 64 + csub;
                int4 v = make_int4(lane, strip, (int)k, acc);
#pragma unroll
                for (int q = 0; q < 16; ++q) *(int4 *)(base + (long)q * 4 * pitch) = v;
                if constexpr (NLOAD > 0) {
#pragma unroll
                    for (int j = 0; j < NLOAD; ++j) acc += ring[ph][j];
                }
                long t0 = clock64();
                while (clock64() - t0 < delay) { }
            }
        }
    }
    if (acc == 0x7fffffff) sink[0] = acc;
}

int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : 131072;
    long pitch = (n + 1 + 63) / 64 * 64;
    long nblocks = (n + 1 + 63) / 64;
    int nstrips = (int)(pitch / 64);
    int *t, *src, *sink;
    if (hipMalloc(&t, (size_t)nblocks * 64 * pitch * 4) != hipSuccess) { printf("oom\n"); return 1; }
    (void)hipMalloc(&src, (1 << 20) * 4 + 4096);
    (void)hipMalloc(&sink, 64);
    (void)hipMemset(src, 1, (1 << 20) * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    auto run = [&](auto kern, const char *name, int waves, int delay) {
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(waves), dim3(64), 0, 0, t, src, pitch, nblocks, nstrips,
                               3L, delay, sink);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
        }
        long done = nblocks / 4 * 4;  // iterations actually run per strip (multiple of DIST+1 <= 4)
        double gbs = (double)(nblocks - nblocks % 4) * 64 * pitch * 4 / (ms * 1e6);
        (void)done;
        // per-wave iteration time implied
        double iters = (double)nstrips * nblocks / waves;
        printf("%-12s waves=%5d delay=%5d ms=%8.3f GB/s=%7.1f us/iter=%.3f\n", name, waves, delay,
               ms, gbs, ms * 1e3 / iters);
    };
    int delays[] = {0, 2000, 3500};
    int wavesv[] = {512, 1024, 2048};
    for (int d : delays)
        for (int w : wavesv) {
            run(cadence<0, 1>, "L0", w, d);
            run(cadence<16, 1>, "L16-D1", w, d);
            run(cadence<16, 3>, "L16-D3", w, d);
            run(cadence<2, 3>, "L2-D3", w, d);
        }
    return 0;
}
