// batch_sweep.hip -- the fill's store pattern, store side only: one workgroup
// per CU sweeps a strip of SW bytes per row top to bottom; its K store waves
// take B-row batches round robin (batch b -> wave b % K), 16 B per lane per
// store (SW = 1024: one row per store; SW = 512: two rows per store).  Strips
// are claimed persistently (strip s by workgroup s % grid), strip s starting at
// row (s * lag) mod nrows and wrapping, so every byte is written exactly once.
// `pace` > 0 makes every wave spin that many cycles per batch (a compute-bound
// producer).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int SW>
__global__ void batch(char *t, long pitchb, long nrows, int K, int B, int nstrips, int lag, int pace) {
    constexpr int R = 1024 / SW;  // rows per store
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int ro = lane / (64 / R), cq = lane % (64 / R);
    typedef unsigned v4 __attribute__((ext_vector_type(4)));
    v4 v = {1u, 2u, 3u, (unsigned)lane};
    for (int s = blockIdx.x; s < nstrips; s += gridDim.x) {
        long r0 = ((long)s * lag) % nrows;
        r0 -= r0 % 64;
        char *base = t + (long)s * SW + (long)ro * pitchb + cq * 16;
        for (long f = (long)wave * B; f < nrows; f += (long)K * B) {
            if (pace) {
                const long long c0 = __builtin_readcyclecounter();
                while (__builtin_readcyclecounter() - c0 < pace) {}
            }
            for (int g = 0; g < B; g += R) {
                long row = f + g + r0;
                if (f + g >= nrows) break;
                if (row >= nrows) row -= nrows;
                *(v4 *)(base + row * pitchb) = v;
                v.x += 1;
            }
        }
    }
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 131072;
    const long extra = argc > 2 ? atol(argv[2]) : 0;  // bytes of row padding
    const long pitchb = n * 4 + extra;
    char *t;
    if (hipMalloc(&t, (size_t)pitchb * n) != hipSuccess) { printf("oom\n"); return 1; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](auto kern, int SW, int K, int B, int grid, int lag, int pace) {
        const int nstrips = (int)(n * 4 / SW);
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * K), 0, 0, t, pitchb, n, K, B, nstrips, lag, pace);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
        }
        const double bytes = (double)n * 4 * n;
        printf("pitch=%ld SW=%4d K=%d B=%2d grid=%4d strips=%4d lag=%4d pace=%4d ms=%7.3f GB/s=%7.1f\n", pitchb, SW, K, B, grid,
               nstrips, lag, pace, ms, bytes / (ms * 1e6));
    };
    if (argc > 3) {
        for (int K : {2, 3, 4}) {
            run(batch<1024>, 1024, K, 16, 256, 192, 0);
            run(batch<512>, 512, K, 16, 256, 192, 0);
        }
        return 0;
    }
    // n = 131072: 512 strips of 1 KB / 1024 of 512 B; grid 256 -> 2 / 4 passes
    for (int K : {1, 2, 3, 4, 6}) {
        run(batch<1024>, 1024, K, 16, 256, 192, 0);
        run(batch<512>, 512, K, 16, 256, 192, 0);
    }
    for (int B : {4, 8, 32, 64}) run(batch<1024>, 1024, 3, B, 256, 192, 0);
    for (int lag : {64, 512, 4096}) run(batch<1024>, 1024, 3, 16, 256, lag, 0);
    // two workgroups per CU
    run(batch<1024>, 1024, 2, 16, 512, 192, 0);
    run(batch<1024>, 1024, 1, 16, 512, 192, 0);
    run(batch<512>, 512, 2, 16, 512, 192, 0);
    return 0;
}
