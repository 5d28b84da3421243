// pass_store.hip -- one pass of the fill's store side (256 workgroups, one 1-KB
// strip each, all rows of a 262144-row, 1-MB-pitch table), to find what sets the
// chip's store rate when the 256 concurrently written strips are neighbours:
// the column spread of the strips (strip b at column offset b * cs KB) and the
// row stagger (strip b starts at row b * lag and wraps).  Stores: 8 rows x 128 B
// per instruction, 4 waves per workgroup owning 256 B each (the fill's (1,4)).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned v4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void pass(char *t, long pitchb, long nrows, int cs, int lag) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x;
    v4 v = {1u, 2u, 3u, (unsigned)lane};
    const long r0 = ((long)b * lag) % nrows;
    const int ro = lane >> 3, cq = lane & 7;
    char *base = t + (long)b * cs * 1024 + wave * 256 + cq * 16;
    for (long f = 0; f < nrows; f += 8) {
        long row = f + ro + r0;
        if (row >= nrows) row -= nrows;
        *(v4 *)(base + row * pitchb) = v;
        *(v4 *)(base + row * pitchb + 128) = v;
        v.x += 1;
    }
}

int main(int argc, char **argv) {
    const long n = 262144;
    const long pitchb = n * 4 + 256;
    char *t;
    if (hipMalloc(&t, (size_t)pitchb * n) != hipSuccess) { printf("oom\n"); return 1; }
    (void)hipMemset(t, 0, (size_t)pitchb * n);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](int cs, int lag, long rows, long roff) {
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            float ms = 0;
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(pass, dim3(256), dim3(256), 0, 0, t + roff * pitchb, pitchb, rows, cs, lag);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep > 0 && ms < best) best = ms;
        }
        const double bytes = (double)rows * 1024.0 * 256;
        printf("cs=%d KB lag=%5d rows=%6ld row0=%6ld ms=%7.3f GB/s=%7.1f ns/row=%.1f\n", cs, lag, rows, roff, best,
               bytes / (best * 1e6), best * 1e6 / rows);
    };
    for (long roff : {0L, 65536L, 196608L}) run(1, 256, 65536, roff);
    for (long rows : {16384L, 32768L, 131072L, 262144L}) run(1, 256, rows, 0);
    run(1, 64, 16384, 0);
    (void)hipFree(t);
    return 0;
}
