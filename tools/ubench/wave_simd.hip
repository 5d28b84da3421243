// wave_simd.hip -- which SIMD does each wave of a workgroup land on (gfx950)?
// Each wave reads HW_REG_HW_ID (SIMD_ID = bits 5:4, CU_ID = bits 11:8) and writes
// it out; printed for workgroups of 1..12 waves, one workgroup per CU (a big LDS
// allocation keeps the others away) and with two per CU.  The strip kernel's
// roles are fixed by wave index (compute waves first, then store waves, then a
// feeder), so the placement decides which waves share a SIMD's issue port.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int LDSB>
__global__ void probe(uint32_t *out) {
    __shared__ char pad[LDSB];
    uint32_t id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = id;
    if (threadIdx.x == 1023) pad[0] = 1;  // (keep the LDS allocation)
    __syncthreads();
    if (threadIdx.x == 1023 && pad[0] == 2) out[0] = 0;
}

int main() {
    uint32_t *d;
    uint32_t h[64 * 16];
    (void)hipMalloc(&d, sizeof h);
    for (int big = 1; big >= 0; --big) {
        printf("== %s\n", big ? "one workgroup per CU (128 KB LDS)" : "small LDS (several per CU)");
        for (int w = 1; w <= 12; ++w) {
            (void)hipMemset(d, 0xFF, sizeof h);
            if (big)
                hipLaunchKernelGGL(probe<131072>, dim3(8), dim3(64 * w), 0, 0, d);
            else
                hipLaunchKernelGGL(probe<64>, dim3(8), dim3(64 * w), 0, 0, d);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
            for (int b = 0; b < 2; ++b) {
                printf("waves=%2d wg %d: simd of wave 0.. =", w, b);
                for (int i = 0; i < w; ++i) printf(" %u", (h[b * 16 + i] >> 4) & 3u);
                printf("   (cu %u)\n", (h[b * 16] >> 8) & 15u);
            }
        }
    }
    return 0;
}
