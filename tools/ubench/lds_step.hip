// lds_step.hip -- what an LDS write per wavefront step costs a compute wave.
// W waves per workgroup (one workgroup per CU), each running the fill's step
// skeleton: a DPP wave_shr:1 left-neighbour shift feeding a dependent chain of
// C v_max3 (C columns per lane), plus the cell adds, then the step's C results
// written to an LDS ring in one of several forms:
//   MODE 0: no LDS write
//   MODE 1: one ds_write_b(32C) per step at a compile-time offset (the fill today)
//   MODE 2: results of 2 steps kept in registers, one ds_write_b(64C) per 2 steps
//   MODE 3: results of 4 steps kept in registers, written per 4 steps (b128 pieces)
// Reports shader cycles per step (s_memtime) of wave 0.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <type_traits>

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

template <int C, int MODE>
__global__ void step(int n, unsigned long long *out, int *sink) {
    __shared__ __attribute__((aligned(16))) char lds[65536];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int u[C];
    for (int k = 0; k < C; ++k) u[k] = lane * 3 + k;
    int dg = lane, s0 = lane * 7, s1 = lane * 5;
    uint32_t base = (uint32_t)wave * 16384u + (uint32_t)lane * (MODE == 3 ? 16u * C : MODE == 2 ? 8u * C : 4u * C);
    asm volatile("" : "+v"(base));
    base &= 0xFFFFu;
    char *ring = lds + base;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        int keep[4][C];
        static_for<0, 16>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            int left = __builtin_amdgcn_update_dpp(s0, u[C - 1], 0x138, 0xF, 0xF, false);
            int diag = dg;
            dg = left;
            static_for<0, C>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                int d;
                asm("v_add_u32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD "
                    "src0_sel:DWORD src1_sel:BYTE_%c3"
                    : "=v"(d)
                    : "v"(diag), "v"(s1), "i"((s + k) & 3));
                const int x = max(max(d, u[k]), left);
                diag = u[k];
                u[k] = x;
                left = x;
                keep[s & 3][k] = x;
            });
            if constexpr (MODE == 1) {
                if constexpr (C == 1) *(int *)(ring + s * 256 * C) = keep[s & 3][0];
                if constexpr (C == 2) *(int2 *)(ring + s * 256 * C) = make_int2(keep[s & 3][0], keep[s & 3][1]);
                if constexpr (C == 4)
                    *(int4 *)(ring + s * 256 * C) = make_int4(keep[s & 3][0], keep[s & 3][1], keep[s & 3][2], keep[s & 3][3]);
            } else if constexpr (MODE == 2 && (s & 1) == 1) {
                if constexpr (C == 1) *(int2 *)(ring + (s / 2) * 512 * C) = make_int2(keep[(s & 3) - 1][0], keep[s & 3][0]);
                if constexpr (C == 2)
                    *(int4 *)(ring + (s / 2) * 512 * C) =
                        make_int4(keep[(s & 3) - 1][0], keep[(s & 3) - 1][1], keep[s & 3][0], keep[s & 3][1]);
            } else if constexpr (MODE == 3 && (s & 3) == 3) {
                if constexpr (C == 1)
                    *(int4 *)(ring + (s / 4) * 1024 * C) = make_int4(keep[0][0], keep[1][0], keep[2][0], keep[3][0]);
                if constexpr (C == 2) {
                    *(int4 *)(ring + (s / 4) * 2048) = make_int4(keep[0][0], keep[0][1], keep[1][0], keep[1][1]);
                    *(int4 *)(ring + (s / 4) * 2048 + 1024) = make_int4(keep[2][0], keep[2][1], keep[3][0], keep[3][1]);
                }
            }
        });
        s1 = s1 * 1103515245 + 12345;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    int acc = dg;
    for (int k = 0; k < C; ++k) acc += u[k];
    if (acc == 0x12345) sink[threadIdx.x] = acc;
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

int main() {
    unsigned long long *d, h[1024];
    int *sink;
    (void)hipMalloc(&d, 1024 * 8);
    (void)hipMalloc(&sink, 4096 * 4);
    const int n = 4096;
    auto run = [&](auto kern, const char *name, int W) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(kern, dim3(256), dim3(64 * W), 0, 0, n, d, sink);
            (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(h, d, 256 * 8, hipMemcpyDeviceToHost);
        double avg = 0;
        for (int i = 0; i < 256; ++i) avg += h[i];
        avg /= 256;
        printf("%-28s waves/CU=%d  cycles/step=%6.1f\n", name, W, avg / (n * 16.0));
    };
    for (int W : {1, 2, 4}) {
        run(step<1, 0>, "C=1 no LDS", W);
        run(step<1, 1>, "C=1 b32 per step", W);
        run(step<1, 2>, "C=1 b64 per 2 steps", W);
        run(step<1, 3>, "C=1 b128 per 4 steps", W);
        run(step<2, 0>, "C=2 no LDS", W);
        run(step<2, 1>, "C=2 b64 per step", W);
        run(step<2, 2>, "C=2 b128 per 2 steps", W);
        run(step<2, 3>, "C=2 2xb128 per 4 steps", W);
        run(step<4, 0>, "C=4 no LDS", W);
        run(step<4, 1>, "C=4 b128 per step", W);
    }
    return 0;
}
