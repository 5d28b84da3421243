// skew_store.hip -- store-only microbenchmark of the fill's HBM write pattern
// WITH the wavefront time skew.  One wave per 64-column strip (like the fill);
// every iteration a wave stores a 64-row x 256-B block (16 x dwordx4, 4 rows per
// instruction) and moves 64 rows down.  Strip p works on rows shifted by
// p*lag (mod the row count), so neighbouring strips touch the same table rows
// `lag` rows apart in time, as in the fill.  Every store stays inside the table.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(64) void skew_store(int *t, long pitch, long nblocks, int nstrips,
                                                 long lag_blocks, int nt) {
    const int strip = blockIdx.x;
    const int lane = threadIdx.x;
    const int rsub = lane >> 4, csub = (lane & 15) * 4;
    int4 v = make_int4(lane, strip, 1, 2);
    long shift = ((long)strip * lag_blocks) % nblocks;
    for (long k = 0; k < nblocks; ++k) {
        long blk = k - shift;
        if (blk < 0) blk += nblocks;
        int *base = t + (blk * 64 + rsub) * pitch + (long)strip * 64 + csub;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            int *p = base + (long)q * 4 * pitch;
            if (nt) {
                typedef int v4i __attribute__((ext_vector_type(4)));
                v4i vv = {v.x, v.y, v.z, v.w};
                __builtin_nontemporal_store(vv, (v4i *)p);
            } else {
                *(int4 *)p = v;
            }
        }
        v.x += 1;
    }
}

int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : 131072;
    long pitch = (n + 1 + 63) / 64 * 64;
    long nblocks = (n + 1 + 63) / 64;
    int nstrips = (int)(pitch / 64);
    int *t;
    if (hipMalloc(&t, (size_t)nblocks * 64 * pitch * 4) != hipSuccess) { printf("oom\n"); return 1; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    long lags[] = {0, 1, 2, 4, 8, 16};  // in 64-row blocks
    for (int nt = 0; nt < 2; ++nt)
        for (long lag : lags) {
            float ms = 0;
            for (int rep = 0; rep < 2; ++rep) {
                (void)hipEventRecord(e0);
                hipLaunchKernelGGL(skew_store, dim3(nstrips), dim3(64), 0, 0, t, pitch, nblocks,
                                   nstrips, lag, nt);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms, e0, e1);
            }
            printf("n=%ld strips=%d lag_rows=%ld nt=%d ms=%.3f GB/s=%.1f\n", n, nstrips, lag * 64,
                   nt, ms, (double)nblocks * 64 * pitch * 4 / (ms * 1e6));
        }
    return 0;
}
