// wide_sweep.hip -- does the HBM store rate of a vertical strip sweep depend on
// how many contiguous bytes of a row one CU writes at about the same time?
// One workgroup of K waves owns a strip of K * PB bytes per row; wave k writes
// bytes [k*PB, (k+1)*PB) of every row (PB = 1 KB: one 16-B-per-lane store per
// row; PB = 512: two rows per store).  The K waves step through the rows in
// lockstep (a workgroup barrier every `sync` rows, 0 = never).  Strips are
// dealt persistently to workgroups, strip s starting at row (s*lag) mod nrows
// (wrapping), so every byte of the table is written once.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void wide(char *t, long pitchb, long nrows, int K, int nstrips, int lag, int sync) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    typedef unsigned v4 __attribute__((ext_vector_type(4)));
    v4 v = {1u, 2u, 3u, (unsigned)lane};
    const long sw = (long)K * 1024;
    for (int s = blockIdx.x; s < nstrips; s += gridDim.x) {
        long r0 = ((long)s * lag) % nrows;
        r0 -= r0 % 64;
        char *base = t + (long)s * sw + wave * 1024 + lane * 16;
        for (long r = 0; r < nrows; ++r) {
            long row = r + r0;
            if (row >= nrows) row -= nrows;
            *(v4 *)(base + row * pitchb) = v;
            v.x += 1;
            if (sync && (r % sync) == sync - 1) __syncthreads();
        }
    }
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 131072;
    const long pitchb = n * 4;  // n columns of int32, a multiple of 8 KB for n % 2048 == 0
    char *t;
    if (hipMalloc(&t, (size_t)pitchb * n) != hipSuccess) { printf("oom\n"); return 1; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](int K, int grid, int lag, int sync) {
        const int nstrips = (int)(pitchb / (K * 1024));
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(wide, dim3(grid), dim3(64 * K), 0, 0, t, pitchb, n, K, nstrips, lag, sync);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
        }
        const double bytes = (double)pitchb * n;
        printf("K=%d (strip %2d KB) grid=%4d lag=%5d sync=%3d ms=%7.3f GB/s=%7.1f\n", K, K, grid, lag, sync, ms,
               bytes / (ms * 1e6));
    };
    for (int K : {1, 2, 4, 8}) {
        run(K, 256, 192, 0);
        run(K, 256, 192, 16);
        run(K, 256, 0, 0);
    }
    run(4, 512, 192, 0);
    run(2, 512, 192, 0);
    run(1, 1024, 192, 0);
    return 0;
}
