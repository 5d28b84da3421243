// strip_store.hip -- store-only microbenchmark of the fill's HBM write pattern.
// Each workgroup owns a vertical strip of W columns and writes it 64 rows at a
// time (row-contiguous segments of W*4 bytes), sweeping down the table, as the
// fill's LDS-ring flush does.  Strips are offset in rows by `lag` per strip
// (the wavefront skew).  Reports achieved GB/s for W in {64,128,256,512}.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int WCOLS>
__global__ __launch_bounds__(256) void strip_store(int *t, long pitch, long nrows, int nstrips,
                                                   int lag, int nt) {
    const int strip = blockIdx.x;
    if (strip >= nstrips) return;
    const int tid = threadIdx.x;
    // each thread stores int4; per instruction the block covers (blockDim*4/WCOLS) rows
    constexpr int kThreads = 256;
    constexpr int kRowsPerInst = kThreads * 4 / WCOLS;
    const int rsub = tid / (WCOLS / 4), csub = (tid % (WCOLS / 4)) * 4;
    int4 v = make_int4(tid, strip, 1, 2);
    // skewed start (negative rows skipped); lag is rounded to a multiple of 64 on
    // the host so every 64-row group lies wholly inside [0, nrows)
    long start = -(long)strip * lag;
    for (long r0 = start; r0 + 64 <= nrows; r0 += 64) {
        if (r0 < 0) continue;
#pragma unroll
        for (int q = 0; q < 64 / kRowsPerInst; ++q) {
            long row = r0 + q * kRowsPerInst + rsub;
            int *p = t + row * pitch + (long)strip * WCOLS + csub;
            typedef int v4i __attribute__((ext_vector_type(4)));
            v4i vv = {v.x, v.y, v.z, v.w};
            if (nt) __builtin_nontemporal_store(vv, (v4i *)p);
            else *(int4 *)p = v;
        }
        v.x += 1;
    }
}

int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : 131072;
    int lag = argc > 2 ? atoi(argv[2]) : 0;
    lag = (lag + 63) / 64 * 64;  // keep 64-row groups aligned (see kernel)
    long pitch = (n + 1 + 63) / 64 * 64;
    long rows = (n + 1 + 63) / 64 * 64;
    int *t;
    if (hipMalloc(&t, (size_t)rows * pitch * 4) != hipSuccess) { printf("oom\n"); return 1; }
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](auto kern, int W, int nt) {
        int nstrips = (int)(pitch / W);
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(nstrips), dim3(256), 0, 0, t, pitch, rows, nstrips, lag, nt);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            if (rep == 2) printf("n=%ld W=%d nt=%d lag=%d strips=%d ms=%.3f GB/s=%.1f\n", n, W, nt, lag,
                                 nstrips, ms, (double)rows * pitch * 4 / (ms * 1e6));
        }
    };
    for (int nt = 0; nt < 2; ++nt) {
        run(strip_store<64>, 64, nt);
        run(strip_store<128>, 128, nt);
        run(strip_store<256>, 256, nt);
        run(strip_store<512>, 512, nt);
        run(strip_store<1024>, 1024, nt);
    }
    // contiguous baseline: one big memset-like pass
    hipEventRecord(e0);
    hipMemsetAsync(t, 1, (size_t)rows * pitch * 4);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("hipMemset GB/s=%.1f\n", (double)rows * pitch * 4 / (ms * 1e6));
    return 0;
}
