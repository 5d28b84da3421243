// fill_store.hip -- the (1,4) fill's store side alone at the bench's scale
// (262144 x 262144 int32, 1 MB pitch, 256 workgroups of 4 store waves, strips of
// 1 KB per row, 4 passes), comparing how the 4 store waves of a strip split it:
//   A "columns": wave w owns the 256-B column piece w of every row (its ring in
//     the fill), 8 rows x 128 B per store instruction (the current fill);
//   B "batches": wave w owns 16-row batches w, w+4, ... and writes whole 1 KB
//     rows, one row per store instruction;
//   C "batches, 512 B": as B, 2 rows x 512 B per instruction (two rings per row half).
// Strip s of a pass starts at row (s * lag) mod nrows and wraps (the fill's
// strips trail each other by one hop), so every byte is written exactly once.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned v4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void sweep(char *t, long pitchb, long nrows, int nstrips, int lag) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    v4 v = {1u, 2u, 3u, (unsigned)lane};
    for (int s = blockIdx.x; s < nstrips; s += gridDim.x) {
        long r0 = ((long)(s % gridDim.x) * lag) % nrows;
        char *sb = t + (long)s * 1024;
        if (MODE == 0 || MODE == 3) {
            // 8 rows x 128 B per instruction, two instructions per 8 rows (64 columns = 256 B);
            // MODE 3: wave w trails wave w-1 by 80 rows (the fill's chained compute waves)
            const int ro = lane >> 3, cq = lane & 7;
            char *base = sb + wave * 256 + cq * 16;
            const long wl = MODE == 3 ? (long)(3 - wave) * 80 : 0;
            for (long f = 0; f < nrows; f += 8) {
                long row = f + ro + r0 + wl;
                if (row >= nrows) row -= nrows;
                if (f + ro >= nrows) continue;
                if (row >= nrows) row -= nrows;
                *(v4 *)(base + row * pitchb) = v;
                *(v4 *)(base + row * pitchb + 128) = v;
                v.x += 1;
            }
        } else if (MODE == 4) {
            // (2,2)-like: waves 0,1 own the left 512 B, waves 2,3 the right 512 B, 16-row
            // batches alternating between the pair, the right pair trailing by 80 rows
            const int ro = lane >> 5, cq = lane & 31;
            const int half = wave >> 1, sub = wave & 1;
            char *base = sb + half * 512 + cq * 16;
            const long wl = (long)(1 - half) * 80;
            for (long f = (long)sub * 16; f < nrows; f += 32) {
                for (int g = 0; g < 16; g += 2) {
                    long row = f + g + ro + r0 + wl;
                    if (f + g + ro >= nrows) break;
                    while (row >= nrows) row -= nrows;
                    *(v4 *)(base + row * pitchb) = v;
                    v.x += 1;
                }
            }
        } else if (MODE == 1) {
            char *base = sb + lane * 16;
            for (long f = (long)wave * 16; f < nrows; f += 64) {
                for (int g = 0; g < 16; ++g) {
                    long row = f + g + r0;
                    if (f + g >= nrows) break;
                    if (row >= nrows) row -= nrows;
                    *(v4 *)(base + row * pitchb) = v;
                    v.x += 1;
                }
            }
        } else {
            const int ro = lane >> 5, cq = lane & 31;
            char *base = sb + cq * 16;
            for (long f = (long)wave * 16; f < nrows; f += 64) {
                for (int g = 0; g < 16; g += 2) {
                    long row = f + g + ro + r0;
                    if (f + g + ro >= nrows) break;
                    if (row >= nrows) row -= nrows;
                    *(v4 *)(base + row * pitchb) = v;
                    *(v4 *)(base + row * pitchb + 512) = v;
                    v.x += 1;
                }
            }
        }
    }
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 262144;
    const long pitchb = n * 4 + 256;
    char *t;
    if (hipMalloc(&t, (size_t)pitchb * n) != hipSuccess) { printf("oom\n"); return 1; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int nstrips = (int)(n * 4 / 1024);
    auto run = [&](auto kern, const char *name, int lag) {
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            float ms = 0;
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, t, pitchb, n, nstrips, lag);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep > 0 && ms < best) best = ms;
        }
        printf("%-22s lag=%4d ms=%7.3f GB/s=%7.1f\n", name, lag, best, (double)n * 4 * n / (best * 1e6));
    };
    // per-CU ceiling: a few workgroups alone (rows limited so a run stays short)
    auto solo = [&](auto kern, const char *name, int grid) {
        const long rows = 65536;
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            float ms = 0;
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, t, pitchb, rows, grid, 256);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep > 0 && ms < best) best = ms;
        }
        const double bytes = (double)rows * 1024.0 * grid;
        printf("%-22s grid=%4d rows=%ld ms=%7.3f GB/s per WG=%6.1f total=%7.1f ns/row=%.1f\n", name, grid, rows,
               best, bytes / (best * 1e6) / grid, bytes / (best * 1e6), best * 1e6 / rows);
    };
    for (int g : {1, 8, 64, 256}) {
        solo(sweep<0>, "A solo", g);
        solo(sweep<1>, "B solo", g);
    }
    for (int lag : {256, 0}) {
        run(sweep<3>, "D columns lagged 80", lag);
        run(sweep<4>, "E halves lagged 80", lag);
        run(sweep<0>, "A columns 8x128B", lag);
        run(sweep<1>, "B batches 1x1KB", lag);
        run(sweep<2>, "C batches 2x512B", lag);
    }
    (void)hipFree(t);
    return 0;
}
