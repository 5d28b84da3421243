// step_loop.hip -- the fill's compute-wave iteration (nw::run_iter) in isolation:
// one compute wave per workgroup, registers and LDS only, N iterations of 64
// steps with every counter already satisfied (no waiting on anyone); reports
// shader cycles per step.  Built against the real kernel source so it times
// exactly the code the fill runs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include \
//         -I../../fast-needleman-wunsch_amd/csrc step_loop.hip -o step_loop
#include "../../fast-needleman-wunsch_amd/csrc/nw_strips.h"

#include <cstdio>

template <int C, int NC, int PUB, int GRAN = 0, int MODE = nw::SUB_PERM>
__global__ __launch_bounds__(64) void step_loop(const uint32_t *pkin, int n, int32_t *out,
                                                unsigned long long *cyc, uint64_t *gsink) {
    typedef nw::Lay<C, NC> L;
    __shared__ __attribute__((aligned(16))) char lds[L::kBytes];
    const int lane = threadIdx.x;
    for (int i = lane; i < L::kBytes / 4; i += 64) ((int32_t *)lds)[i] = 0;
    int32_t *ctr = (int32_t *)(lds + L::kCtl);
    __syncthreads();
    if (lane == 0) {
        for (int q = 0; q < L::kSPR; ++q) ctr[3 + q] = nw::kDone;  // ring always free
    }
    __syncthreads();
    nw::Lanes<C> S;
    S.apk = 0x01020304u * (lane & 3);
#pragma unroll
    for (int k = 0; k < C; ++k) {
        S.u[k] = lane + k;
        S.tlo[k] = 0x01000100u + k;
        S.thi[k] = 0x00010001u;
    }
    S.dg = 0;
    S.rr = 0;
    S.cb = nw::kDone;
    S.rcol = 0;
    S.rb[0] = (uint32_t)lane * (4u * C);
    S.rb[1] = S.rb[0] + 64u * L::kSlot;
    S.rc[0] = S.rc[1] = (uint32_t)((lane & 15) * L::kSlot);
    S.z = lane;
    S.psel = false;
    S.pofs = 0;
    S.pbase = 0;
    nw::Feed F;
    F.src = nw::FEED_LDS;
    F.ring = (int32_t *)(lds + L::kFeed);
    F.pub = ctr + 1;
    F.tag = 0;
    F.ready = 4;
    F.gap = -1;
    F.nslow = 0;
    F.wticks = 0;
    F.rticks = 0;
    F.dead = false;
    F.trace_pub = false;
    F.tpub = 0;
    F.tmo = 100000000ull * 20ull;
    nw::Out O;
    O.off = false;
    O.lds = !GRAN;
    O.ring = (int32_t *)(lds + L::kFeed) + (NC > 1 ? nw::kFeedRows : 0);
    O.pub = ctr + 9;
    O.gap = -1;
    nw::u32x4 pk[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) pk[h] = ((const nw::u32x4 *)pkin)[lane * 4 + h];
    uint32_t ctrl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 1; it <= n; it += 2) {
        nw::run_iter<C, NC, MODE, false, 1>(lds, it, pk, 2, 1, -1, S, ctr, ctr + 3,
                                                    PUB ? it - 1 : -1, gsink + blockIdx.x * 64 + lane, 0, O, ctrl, F, lane);
        nw::run_iter<C, NC, MODE, false, 0>(lds, it + 1, pk, 2, 1, -1, S, ctr, ctr + 3,
                                                    PUB ? it : -1, gsink + blockIdx.x * 64 + lane, 0, O, ctrl, F, lane);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + lane] = S.u[0] + S.rcol;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    uint32_t *pk;
    int32_t *out;
    unsigned long long *cyc, h[1024];
    uint64_t *gs;
    (void)hipMalloc(&pk, 64 * 64);
    (void)hipMemset(pk, 1, 64 * 64);
    (void)hipMalloc(&out, 1024 * 256);
    (void)hipMalloc(&cyc, 8 * 1024);
    (void)hipMalloc(&gs, 1024 * 64 * 8);
    const int n = 2000;
    auto run = [&](auto kern, const char *name, int grid) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, pk, n, out, cyc, gs);
            (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(h, cyc, 8 * grid, hipMemcpyDeviceToHost);
        double avg = 0;
        for (int i = 0; i < grid; ++i) avg += h[i];
        avg /= grid;
        printf("%-20s grid=%4d cycles/step %.1f\n", name, grid, avg / (n * 64.0));
    };
    for (int grid : {1, 256}) {
        run(step_loop<2, 2, 1>, "C=2 NC=2 publish", grid);
        run(step_loop<2, 2, 0>, "C=2 NC=2 no publish", grid);
        run(step_loop<2, 2, 1, 1>, "C=2 NC=2 granules", grid);
        run(step_loop<1, 4, 1>, "C=1 NC=4 publish", grid);
        run(step_loop<4, 1, 1>, "C=4 NC=1 publish", grid);
        run(step_loop<2, 2, 1, 1, nw::SUB_PERM_SW>, "SW C=2 NC=2 granules", grid);
        run(step_loop<2, 2, 1, 0, nw::SUB_PERM_SW>, "SW C=2 NC=2 publish", grid);
        run(step_loop<4, 1, 1, 1, nw::SUB_PERM_SW>, "SW C=4 NC=1 granules", grid);
    }
    return 0;
}
