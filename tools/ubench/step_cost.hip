// step_cost.hip -- cycles per wavefront step of the NW recurrence on gfx950,
// with components switched on/off, one wave per SIMD (4 per CU), to find what
// bounds the fill kernel's inner loop.
//   LDS : write t to the 128-row LDS ring ((base + 256u) & 0x7FFF, ds_write_b32)
//   DPP : left via DPP wave_shr:1 (else a plain copy: no cross-lane)
//   CMP : 0 = v_cmp_eq_u32_sdwa + v_addc (UNIT), 1 = sdwa cmp + v_cndmask, 2 = none
//   K   : independent chains interleaved per step
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o step_cost step_cost.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <type_traits>

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

template <int Q, int CMP>
__device__ __forceinline__ int32_t diag(uint32_t pk, uint32_t a, int32_t tl, int32_t msp, int32_t mmp) {
    if constexpr (CMP == 2) return tl + mmp;
    int32_t d;
    if constexpr (CMP == 0) {
        asm volatile("v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_%5 src1_sel:DWORD\n"
                     "v_addc_co_u32_e32 %0, vcc, %3, %4, vcc"
                     : "=v"(d) : "v"(pk), "v"(a), "v"(tl), "v"(mmp), "i"(Q) : "vcc");
    } else {
        int32_t s;
        asm volatile("v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_%5 src1_sel:DWORD\n"
                     "v_cndmask_b32_e32 %0, %3, %4, vcc"
                     : "=v"(s) : "v"(pk), "v"(a), "v"(mmp), "v"(msp), "i"(Q) : "vcc");
        d = tl + s;
    }
    return d;
}

template <int K, int LDS, bool DPP, int CMP>
__global__ __launch_bounds__(64) void steps(int iters, int32_t gap, int32_t *out, uint64_t *cyc) {
    __shared__ __attribute__((aligned(16))) int32_t ring[K * 128 * 64];
    const int lane = threadIdx.x;
    int32_t tg[K], tl[K];
    uint32_t a[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        tg[k] = lane * 3 + k;
        tl[k] = lane;
        a[k] = (lane * 7 + k) & 3;
    }
    uint32_t pk = 0x01020304u * (lane & 3);
    uint32_t laddr = ((uint32_t)(-1 - lane) & 127u) * 256u + (uint32_t)lane * 4u;
    const int32_t msp = 1 - gap, mmp = 0 - gap;
    int32_t tprev[K], tprev2[K];
    uint32_t offprev = laddr, offprev2 = laddr;
#pragma unroll
    for (int k = 0; k < K; ++k) tprev[k] = tprev2[k] = 0;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        asm volatile("" : "+v"(laddr), "+v"(pk));
        static_for<0, 64>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            uint32_t off;
            if constexpr (LDS == 1 || LDS == 0 || LDS == 5 || LDS == 6) off = (laddr + 256u * (uint32_t)(u + 1)) & 0x7FFFu;
            if constexpr (LDS == 2) off = (laddr + 256u * (uint32_t)(u + 1));
            if constexpr (LDS == 3) off = (laddr & 0x40FCu) + 256u * (uint32_t)u;  // slot row u (+parity), word = lane
            if constexpr (LDS == 4) off = (uint32_t)lane * 4u;
            const uint32_t offp = offprev, offp2 = offprev2;
            static_for<0, K>([&](auto kk) {
                constexpr int k = K - 1 - decltype(kk)::value;
                const uint32_t offprev = offp, offprev2 = offp2;
                (void)offprev; (void)offprev2;
                int32_t lf = k == 0 ? u : tg[k == 0 ? 0 : k - 1];
                int32_t tln;
                if constexpr (DPP) tln = __builtin_amdgcn_update_dpp(lf, tg[k], 0x138, 0xF, 0xF, false);
                else tln = tg[k] ^ lf;
                const int32_t d = diag<u & 3, CMP>(pk, a[k], tl[k], msp, mmp);
                const int32_t t = max(max(d, tg[k]), tln);
                tg[k] = t + gap;
                tl[k] = tln;
                if constexpr (LDS == 5) {  // write the previous step's value
                    *(int32_t *)((char *)ring + k * 32768 + offprev) = tprev[k];
                    tprev[k] = t;
                } else if constexpr (LDS == 6) {  // two steps late
                    *(int32_t *)((char *)ring + k * 32768 + offprev2) = tprev2[k];
                    tprev2[k] = tprev[k];
                    tprev[k] = t;
                } else if constexpr (LDS != 0) {
                    *(int32_t *)((char *)ring + k * 32768 + off) = t;
                }
            });
            offprev2 = offprev;
            offprev = off;
        });
        laddr ^= 64u * 256u;
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    int32_t acc = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) acc += tg[k] + tl[k];
    if (LDS != 0) acc += ring[lane * 64 + 3];
    out[blockIdx.x * 64 + lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = c1 - c0;
}

template <int K, int LDS, bool DPP, int CMP>
void run(const char *name, int32_t *out, uint64_t *cyc, int grid, int iters) {
    hipLaunchKernelGGL((steps<K, LDS, DPP, CMP>), dim3(grid), dim3(64), 0, 0, 1, -1, out, cyc);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((steps<K, LDS, DPP, CMP>), dim3(grid), dim3(64), 0, 0, iters, -1, out, cyc);
    hipEventRecord(e1);
    hipDeviceSynchronize();
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    uint64_t c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double steps = 64.0 * iters;
    printf("%-34s grid %5d: %6.1f clk/step (s_memtime)  %6.2f ns/step (event)  -> %6.1f clk/step/chain\n",
           name, grid, c / steps, ms * 1e6 / steps, c / steps / K);
}

int main() {
    int32_t *out;
    uint64_t *cyc;
    const int maxg = 2048;
    hipMalloc(&out, maxg * 64 * 4);
    hipMalloc(&cyc, maxg * 8);
    const int iters = 4000;
    for (int grid : {1024}) {
        run<1, 1, true, 0>("K1 lds-skew+and dpp cmp (kernel)", out, cyc, grid, iters);
        run<1, 5, true, 0>("K1 lds-skew+and DELAY1 dpp cmp", out, cyc, grid, iters);
        run<1, 6, true, 0>("K1 lds-skew+and DELAY2 dpp cmp", out, cyc, grid, iters);
        run<1, 0, true, 0>("K1 nolds dpp cmp", out, cyc, grid, iters);
        run<2, 1, true, 0>("K2 lds-skew+and dpp cmp (kernel)", out, cyc, grid, iters);
        run<2, 5, true, 0>("K2 lds-skew+and DELAY1 dpp cmp", out, cyc, grid, iters);
        run<2, 6, true, 0>("K2 lds-skew+and DELAY2 dpp cmp", out, cyc, grid, iters);
        run<2, 0, true, 0>("K2 nolds dpp cmp", out, cyc, grid, iters);
        run<4, 5, true, 0>("K4 lds-skew+and DELAY1 dpp cmp", out, cyc, grid, iters);
    }
    return 0;
}
