// pingpong.hip -- hand-off round-trip latency between two waves on MI355X.
//
// WG 0 and WG `peer` bounce a counter through two 8-byte words; the other WGs
// optionally stream 1 KiB stores (global_store_dwordx4 x 64 lanes) to load HBM
// like the fill kernel does.  Modes (how the flag words are stored/loaded):
//   0: agent-scope relaxed atomics   (what nw_fill uses: sc1)
//   1: L2-coherent only              (inline asm: load sc0 / store sc0)
//   2: system-scope relaxed atomics  (sc0 sc1)
// Prints the round-trip time and the XCC ids of the two WGs.
// Build: hipcc --offload-arch=gfx950 -O3 -o pingpong pingpong.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr uint64_t kTimeout = 100000000ull * 2;  // 2 s at 100 MHz

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v;
}

template <int MODE>
__device__ __forceinline__ uint64_t ld(uint64_t *p) {
    if constexpr (MODE == 0) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (MODE == 2) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint64_t v;
    asm volatile("global_load_dwordx2 %0, %1, off sc0\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
template <int MODE>
__device__ __forceinline__ void st(uint64_t *p, uint64_t v) {
    if constexpr (MODE == 0) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); return; }
    if constexpr (MODE == 2) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); return; }
    asm volatile("global_store_dwordx2 %0, %1, off sc0" : : "v"(p), "v"(v) : "memory");
}

template <int MODE>
__global__ __launch_bounds__(64) void pingpong(uint64_t *flags, uint32_t *info, int peer, int rounds,
                                               int4 *bg, int64_t bg_words_per_wg, int bg_on) {
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    uint32_t *stop = info + 8;
    if (b == 0 || b == peer) {
        if (lane == 0) info[b == 0 ? 0 : 1] = xcc_id();
        uint64_t *mine = flags + (b == 0 ? 0 : 16);   // separate 128-B lines
        uint64_t *theirs = flags + (b == 0 ? 16 : 0);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool dead = false;
        for (int k = 1; k <= rounds && !dead; ++k) {
            if (b == 0) st<MODE>(mine, (uint64_t)k);
            for (;;) {
                const uint64_t v = ld<MODE>(theirs);
                if (v >= (uint64_t)k) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeout) { dead = true; break; }
            }
            if (b != 0) st<MODE>(mine, (uint64_t)k);
        }
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        if (b == 0 && lane == 0) {
            info[2] = (uint32_t)(t1 - t0);
            info[3] = dead;
            __hip_atomic_store(stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    if (!bg_on) return;
    // background: stream 1 KiB stores round-robin through this WG's slice
    int4 *base = bg + (int64_t)b * bg_words_per_wg;
    const int4 v = make_int4(b, lane, 1, 2);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int64_t it = 0;; ++it) {
#pragma unroll
        for (int u = 0; u < 16; ++u) base[((it * 16 + u) * 64 + lane) % bg_words_per_wg] = v;
        if (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeout) break;
    }
}

int main(int argc, char **argv) {
    const int rounds = 2000;
    const int grid = 1024;
    const int64_t per_wg = 1 << 16;  // int4 per background WG = 1 MiB
    uint64_t *flags;
    uint32_t *info;
    int4 *bg;
    hipMalloc(&flags, 4096);
    hipMalloc(&info, 64);
    if (hipMalloc(&bg, (size_t)grid * per_wg * sizeof(int4)) != hipSuccess) { printf("oom\n"); return 1; }
    int peers[] = {1, 2, 4, 8, 16, 9};
    for (int bgon = 0; bgon <= 1; ++bgon)
        for (int mode = 0; mode <= 2; ++mode)
            for (int peer : peers) {
                hipMemset(flags, 0, 4096);
                hipMemset(info, 0, 64);
                if (mode == 0)
                    hipLaunchKernelGGL(pingpong<0>, dim3(grid), dim3(64), 0, 0, flags, info, peer, rounds, bg, per_wg, bgon);
                else if (mode == 1)
                    hipLaunchKernelGGL(pingpong<1>, dim3(grid), dim3(64), 0, 0, flags, info, peer, rounds, bg, per_wg, bgon);
                else
                    hipLaunchKernelGGL(pingpong<2>, dim3(grid), dim3(64), 0, 0, flags, info, peer, rounds, bg, per_wg, bgon);
                hipEvent_t e0, e1;
                hipEventCreate(&e0);
                hipEventCreate(&e1);
                hipDeviceSynchronize();
                uint32_t h[4];
                hipMemcpy(h, info, 16, hipMemcpyDeviceToHost);
                printf("bg=%d mode=%d peer=%2d xcc %u/%u  rtt %.3f us%s\n", bgon, mode, peer, h[0], h[1],
                       h[2] / 100.0 / rounds, h[3] ? "  TIMEOUT" : "");
                fflush(stdout);
            }
    hipFree(bg);
    hipFree(flags);
    hipFree(info);
    return 0;
}
