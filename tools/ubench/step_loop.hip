// step_loop.hip -- the fill's compute-wave iteration (nw::run_iter) in isolation:
// one wave, registers and LDS only, N iterations of 64 steps; reports shader
// cycles per step.  Built against the real kernel source so it times exactly
// the code the fill runs.
//   hipcc --offload-arch=gfx950 -O3 -I../../include -I../../fast-needleman-wunsch_amd/csrc step_loop.hip
#include "../../fast-needleman-wunsch_amd/csrc/nw_fill.hip"

#include <cstdio>

template <int C>
__global__ __launch_bounds__(64) void step_loop(const uint32_t *pkin, int n, int32_t *out,
                                                unsigned long long *cyc, uint64_t *gsink) {
    typedef nw::Lay<C> L;
    __shared__ __attribute__((aligned(16))) char lds[L::kBytes];
    const int lane = threadIdx.x;
    for (int i = lane; i < L::kBytes / 4; i += 64) ((int32_t *)lds)[i] = 0;
    int32_t *ctr = (int32_t *)(lds + L::kCtl);
    if (lane == 0) ctr[1] = nw::kDone;
    __syncthreads();
    nw::Lanes<C> S;
    S.apk = 0x01020304u * (lane & 3);
#pragma unroll
    for (int k = 0; k < C; ++k) S.u[k] = lane + k;
    S.dg = 0;
    S.rr = 0;
    S.outcol = 0;
    S.cb = nw::kDone;
    nw::u32x4 pk[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) pk[h] = ((const nw::u32x4 *)pkin)[lane * 4 + h];
    uint32_t ctrl[4] = {0, 0, 0, 0};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 1; it <= n; ++it) {
        const int sb = __builtin_amdgcn_readfirstlane((int)(((uint32_t)it * 64u) % (uint32_t)L::R));
        nw::run_iter<C, true, false>(lds, it, pk, 2, 1, -1, S, sb, gsink + lane, 0, ctrl, lane);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = S.u[0] + S.outcol;
    if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
    uint32_t *pk;
    int32_t *out;
    unsigned long long *cyc, h;
    uint64_t *gs;
    (void)hipMalloc(&pk, 64 * 64);
    (void)hipMemset(pk, 1, 64 * 64);
    (void)hipMalloc(&out, 256);
    (void)hipMalloc(&cyc, 8);
    (void)hipMalloc(&gs, 64 * 8);
    const int n = 2000;
    auto run = [&](auto kern, int c) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, pk, n, out, cyc, gs);
            (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("C=%d cycles/step %.1f  cycles/cell %.3f\n", c, (double)h / (n * 64.0),
               (double)h / (n * 64.0 * 64 * c));
    };
    run(step_loop<1>, 1);
    run(step_loop<2>, 2);
    run(step_loop<4>, 4);
    return 0;
}
