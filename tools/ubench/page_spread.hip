// page_spread.hip -- HBM store rate of 128-byte row pieces as a function of how
// many table rows (each its own 2 MB page at config 4's pitch) are written at once.
// The horizontal strips of a row band write 128-byte pieces of ALL the band's
// 65536 rows as they sweep the columns; the vertical strips and the panels write
// a few hundred rows at a time.  256 workgroups (one per CU) x 4 waves; workgroup
// b owns rows b*R .. b*R+R-1 and sweeps its rows' first `span` bytes in 128-byte
// column batches, writing every one of its R rows per batch (one store instruction
// = 8 rows x 128 B, the store_strip_tr shape).  R = 8 .. 256 => 2048 .. 65536 rows
// (pages) in flight.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void pieces(char *base, long pitch, int R, long span) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ro = lane >> 3, pc = lane & 7;  // row within the 8-row group, 16-B piece
    const long row0 = (long)blockIdx.x * R;
    const int ngroups = (R + 7) / 8;
    u32x4 v = {(uint32_t)lane, (uint32_t)blockIdx.x, 1u, 2u};
    for (long x = 0; x < span; x += 128) {
        for (int g = wave; g < ngroups; g += 4) {
            const int r = g * 8 + ro;
            if (r < R) *(u32x4 *)(base + (row0 + r) * pitch + x + pc * 16) = v;
        }
        v.x += 1u;
    }
}

int main() {
    const long pitch = 2097408;  // 524288 + 64 columns of int32 (config 4's band row pitch, 256-B aligned)
    const long rows_max = 65536;
    char *t;
    if (hipMalloc(&t, pitch * rows_max) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int R : {8, 16, 32, 64, 128, 256}) {
        const long rows = 256L * R;
        long span = (8L << 30) / rows;  // ~8 GB per run
        span = span / 128 * 128;
        if (span > pitch - 256) span = (pitch - 256) / 128 * 128;
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(pieces, dim3(256), dim3(256), 0, 0, t, pitch, R, span);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        const double bytes = (double)rows * span;
        printf("rows in flight %6ld (R=%3d per CU), %7ld B per row: %7.3f ms, %7.1f GB/s\n", rows, R, span, best,
               bytes / (best * 1e6));
    }
    return 0;
}
