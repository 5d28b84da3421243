// cu_store.hip -- is the vector-store issue path a per-CU or a per-SIMD resource?
// One workgroup of W waves (so all W waves share one CU, one per SIMD up to 4)
// issues N back-to-back stores per wave, each a whole row segment (64 lanes x
// 4/8/16 B) into rows `pitch` bytes apart (the fill's pattern).  Reports bytes
// per shader cycle for the CU.  A second mode runs the same on every CU
// (grid = 256 * copies) for the chip-wide rate.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int DW>
__global__ void store_rows(char *t, long pitch, int n, long wgstride, unsigned long long *cyc) {
    typedef int v4 __attribute__((ext_vector_type(4)));
    typedef int v2 __attribute__((ext_vector_type(2)));
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    char *base = t + (long)blockIdx.x * wgstride + (long)wave * (64 * DW * 4) + lane * DW * 4;
    const unsigned long long c0 = __builtin_readcyclecounter();
    v4 x = {lane, wave, 1, 2};
    for (int i = 0; i < n; ++i) {
        char *p = base + (long)i * pitch;
        if constexpr (DW == 4) *(v4 *)p = x;
        else if constexpr (DW == 2) *(v2 *)p = (v2){x.x, x.y};
        else *(int *)p = x.x;
        x.x += 1;
    }
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long c1 = __builtin_readcyclecounter();
    if (lane == 0) cyc[blockIdx.x * 16 + wave] = c1 - c0;
}

int main(int argc, char **argv) {
    const long pitch = 1 << 20;  // 1 MiB between rows (256k-column table)
    const int n = 4096;
    char *t;
    unsigned long long *cyc;
    size_t bytes = (size_t)pitch * n + (64 << 20);
    if (hipMalloc(&t, bytes) != hipSuccess) return 1;
    (void)hipMalloc(&cyc, 256 * 64 * 16 * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    unsigned long long h[64 * 16];
    auto run = [&](auto kern, int dw, int waves, int grid, const char *tag) {
        // wgstride: workgroups write disjoint column ranges of the same rows
        long wgstride = (long)waves * 64 * dw * 4;
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), 0, 0, t, pitch, n, wgstride, cyc);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
        }
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipMemcpy(h, cyc, sizeof(unsigned long long) * 16 * (grid < 64 ? grid : 64), hipMemcpyDeviceToHost);
        double totb = (double)grid * waves * n * 64 * dw * 4;
        printf("%-6s DW=%d waves/WG=%2d grid=%4d  cycles(wave0)=%8llu  B/cyc/CU(wave0 view)=%6.2f  "
               "cyc/store/wave=%6.1f  chip GB/s=%8.1f\n", tag, dw, waves, grid, h[0],
               (double)waves * n * 64 * dw * 4 / (double)h[0], (double)h[0] / n, totb / (ms * 1e6));
    };
    for (int w : {1, 2, 3, 4, 8}) {
        run(store_rows<4>, 4, w, 1, "1CU");
        run(store_rows<2>, 2, w, 1, "1CU");
        run(store_rows<1>, 1, w, 1, "1CU");
    }
    for (int w : {1, 2, 4}) {
        run(store_rows<4>, 4, w, 256, "chip");
        run(store_rows<4>, 4, w, 512, "chip");
    }
    // how many storing CUs saturate HBM (one workgroup per CU while grid <= 256)
    for (int w : {4, 8})
        for (int g : {32, 64, 96, 128, 160, 192, 224, 256}) run(store_rows<4>, 4, w, g, "ncu");
    return 0;
}
