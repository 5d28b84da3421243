// store_shape.hip -- chip-wide HBM store rate of a strip sweep as a function of
// the SHAPE of one store instruction.  Each storing wave owns a vertical strip
// of SW bytes per row and sweeps it top to bottom (rotated start: strip s
// begins at row (s * lag) mod nrows and wraps, so every byte of the table is
// written exactly once), R rows per 16-byte-per-lane store instruction
// (R rows x 1024/R bytes; R = 1024/SW covers the whole strip width).
// Strips are dealt to waves persistently.  The fill's store waves today issue
// R = 2 (two 512-B ring rows per instruction).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int R, int NT>
__global__ void sweep(char *t, long pitchb, long nrows, int sw, int nstrips, int lag, int idle) {
    constexpr int LPR = 64 / R;  // lanes per row of one instruction
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    if (wave < idle) return;
    const int wpg = blockDim.x / 64 - idle;
    const int wid = blockIdx.x * wpg + (wave - idle);
    const int nw = gridDim.x * wpg;
    const int ro = lane / LPR, cq = lane % LPR;
    const int pieces = sw / (LPR * 16);  // instructions per R rows
    typedef unsigned v4 __attribute__((ext_vector_type(4)));
    v4 v = {1u, 2u, 3u, (unsigned)lane};
    for (int s = wid; s < nstrips; s += nw) {
        long r0 = ((long)s * lag) % nrows;
        r0 -= r0 % 64;
        char *base = t + (long)s * sw + (long)ro * pitchb + cq * 16;
        for (long r = 0; r < nrows; r += R) {
            long row = r + r0;
            if (row >= nrows) row -= nrows;
            for (int k = 0; k < pieces; ++k) {
                v4 *p = (v4 *)(base + row * pitchb + k * (LPR * 16));
                if constexpr (NT) __builtin_nontemporal_store(v, p);
                else *p = v;
            }
            v.x += 1;
        }
    }
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 65536;  // rows; columns = n as well
    const long pitchb = ((n + 64) / 64 * 64 + 64) * 4;
    char *t;
    if (hipMalloc(&t, (size_t)pitchb * (n + 64)) != hipSuccess) { printf("oom\n"); return 1; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](auto kern, int R, int nt, int sw, int grid, int wpb, int idle, int lag) {
        const int nstrips = (int)(n * 4 / sw);
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * wpb), 0, 0, t, pitchb, n, sw, nstrips, lag, idle);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
        }
        const double bytes = (double)nstrips * sw * n;
        printf("SW=%5d R=%2d nt=%d grid=%4d waves/WG=%d idle=%d storing=%5d lag=%4d ms=%7.3f GB/s=%7.1f\n", sw,
               R, nt, grid, wpb, idle, grid * (wpb - idle), lag, ms, bytes / (ms * 1e6));
    };
    const int lag = 192;
    // the fill today: 512-B strips (C = 2 rings), 4 storing waves per CU
    for (int sw : {512, 1024}) {
        run(sweep<1, 0>, 1, 0, sw, 256, 6, 2, lag);
        run(sweep<2, 0>, 2, 0, sw, 256, 6, 2, lag);
        run(sweep<4, 0>, 4, 0, sw, 256, 6, 2, lag);
        run(sweep<8, 0>, 8, 0, sw, 256, 6, 2, lag);
        run(sweep<16, 0>, 16, 0, sw, 256, 6, 2, lag);
        run(sweep<4, 1>, 4, 1, sw, 256, 6, 2, lag);
        run(sweep<8, 1>, 8, 1, sw, 256, 6, 2, lag);
    }
    // storing waves per CU at R = 4 / 8
    for (int w : {1, 2, 3, 4, 6, 8}) {
        run(sweep<4, 0>, 4, 0, 512, 256, w + 2, 2, lag);
        run(sweep<8, 0>, 8, 0, 512, 256, w + 2, 2, lag);
    }
    // 256-B strips
    run(sweep<4, 0>, 4, 0, 256, 256, 6, 2, lag);
    run(sweep<8, 0>, 8, 0, 256, 256, 6, 2, lag);
    run(sweep<16, 0>, 16, 0, 256, 256, 6, 2, lag);
    // lag sensitivity at R = 8
    for (int lg : {0, 64, 1024, 8192}) run(sweep<8, 0>, 8, 0, 512, 256, 6, 2, lg);
    return 0;
}
