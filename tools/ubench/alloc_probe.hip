// alloc_probe.hip -- store rate of the fill's one-pass strip pattern (256 x 1 KB
// strips, 1 MB pitch, 16384-row windows) at different offsets into allocations,
// to map which parts of a large allocation write slowly.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned v4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void pass(char *t, long pitchb, long nrows, int lag) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x;
    v4 v = {1u, 2u, 3u, (unsigned)lane};
    const long r0 = ((long)b * lag) % nrows;
    const int ro = lane >> 3, cq = lane & 7;
    char *base = t + (long)b * 1024 + wave * 256 + cq * 16;
    for (long f = 0; f < nrows; f += 8) {
        long row = f + ro + r0;
        if (row >= nrows) row -= nrows;
        *(v4 *)(base + row * pitchb) = v;
        *(v4 *)(base + row * pitchb + 128) = v;
        v.x += 1;
    }
}

// one 1-KB row per store instruction (4 waves take 16-row batches round robin)
__global__ __launch_bounds__(256) void pass_rows(char *t, long pitchb, long nrows, int lag) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x;
    v4 v = {1u, 2u, 3u, (unsigned)lane};
    const long r0 = ((long)b * lag) % nrows;
    char *base = t + (long)b * 1024 + lane * 16;
    for (long f = (long)wave * 16; f < nrows; f += 64)
        for (int g = 0; g < 16; ++g) {
            long row = f + g + r0;
            if (row >= nrows) row -= nrows;
            *(v4 *)(base + row * pitchb) = v;
            v.x += 1;
        }
}

// strips spread over an allocation of `total` rows: strip b writes `rows` rows from row b * lag
__global__ __launch_bounds__(256) void pass_span(char *t, long pitchb, long total, long rows, int lag) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x;
    v4 v = {1u, 2u, 3u, (unsigned)lane};
    const long r0 = ((long)b * lag) % total;
    const int ro = lane >> 3, cq = lane & 7;
    char *base = t + (long)b * 1024 + wave * 256 + cq * 16;
    for (long f = 0; f < rows; f += 8) {
        long row = f + ro + r0;
        if (row >= total) row -= total;
        *(v4 *)(base + row * pitchb) = v;
        *(v4 *)(base + row * pitchb + 128) = v;
        v.x += 1;
    }
}

static hipEvent_t e0, e1;
static void probe_rows(const char *name, char *t, long pitchb, long roff, long rows) {
    float best = 1e9f;
    for (int rep = 0; rep < 3; ++rep) {
        float ms = 0;
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(pass_rows, dim3(256), dim3(256), 0, 0, t + roff * pitchb, pitchb, rows, 64);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0 && ms < best) best = ms;
    }
    printf("%-10s GB-offset=%6.1f rows=%ld ms=%6.3f GB/s=%7.1f (1 row per store)\n", name, roff * (double)pitchb / 1e9,
           rows, best, (double)rows * 1024.0 * 256 / (best * 1e6));
}
static void probe(const char *name, char *t, long pitchb, long roff, long rows) {
    float best = 1e9f;
    for (int rep = 0; rep < 3; ++rep) {
        float ms = 0;
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(pass, dim3(256), dim3(256), 0, 0, t + roff * pitchb, pitchb, rows, 64);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0 && ms < best) best = ms;
    }
    printf("%-10s GB-offset=%6.1f rows=%ld ms=%6.3f GB/s=%7.1f\n", name, roff * (double)pitchb / 1e9, rows, best,
           (double)rows * 1024.0 * 256 / (best * 1e6));
}

int main() {
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const long pitchb = 262144L * 4 + 256;
    char *small = nullptr, *big = nullptr;
    (void)hipMalloc(&small, (size_t)pitchb * 16384);
    (void)hipMemset(small, 0, (size_t)pitchb * 16384);
    probe("small16G", small, pitchb, 0, 16384);
    const long brows = 200000;
    if (hipMalloc(&big, (size_t)pitchb * brows) != hipSuccess) { printf("oom\n"); return 1; }
    (void)hipMemset(big, 0, (size_t)pitchb * brows);
    for (long r = 0; r + 16384 <= brows; r += 3 * 16384) probe("big200G", big, pitchb, r, 16384);
    // the same bytes (256 strips x 16384 rows) but the strips spread over the
    // whole allocation: strip b starts at row b * 781 and wraps over all rows
    {
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            float ms = 0;
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(pass_span, dim3(256), dim3(256), 0, 0, big, pitchb, brows, 16384L, 781);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep > 0 && ms < best) best = ms;
        }
        printf("spread over 200G: ms=%6.3f GB/s=%7.1f\n", best, 16384.0 * 1024.0 * 256 / (best * 1e6));
    }
    (void)hipFree(small);
    (void)hipFree(big);
    big = nullptr;
    hipError_t e = hipExtMallocWithFlags((void **)&big, (size_t)pitchb * brows, hipDeviceMallocContiguous);
    printf("contiguous alloc: %s\n", hipGetErrorString(e));
    if (e == hipSuccess) {
        (void)hipMemset(big, 0, (size_t)pitchb * brows);
        for (long r = 0; r + 16384 <= brows; r += 3 * 16384) probe("contig200G", big, pitchb, r, 16384);
        (void)hipFree(big);
    }
    return 0;
}
