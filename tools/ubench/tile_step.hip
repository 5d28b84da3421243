// tile_step.hip -- cycles per wavefront step when a lane computes an R x C TILE
// (R consecutive rows x C consecutive columns) of the NW recurrence per step
// instead of one row of C columns (the strip kernel, R = 1).  w form:
//   x = max3(w_diag + s', w_up, w_left)
// Per step a lane takes its left column (R values) from lane l-1's right column of
// the previous step (R DPP wave_shr:1), computes the tile in anti-diagonal order
// and writes it to an LDS ring slot (R*C int32 per lane).  The row chain through a
// step is R max3 (the up dependency), the left chain C max3 + one DPP -- a step
// advances R rows, so the rows-per-time of a strip grows with R while the
// columns-per-step of the lane skew stays C.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tile_step tile_step.hip
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

template <int R, int C>
__global__ __launch_bounds__(64) void steps(int iters, int32_t *out, uint64_t *cyc) {
    constexpr int kSlot = 64 * R * C * 4;  // bytes per ring slot
    __shared__ __attribute__((aligned(16))) char ring[16 * kSlot];
    const int lane = threadIdx.x;
    int32_t u[C], rc[R];
    uint32_t tlo[C], thi[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        u[c] = lane + c;
        tlo[c] = 0x01FF01FFu * (uint32_t)((lane + c) & 1);
        thi[c] = 0xFF01FF01u;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) rc[r] = lane - r;
    int32_t dg = 0;
    uint32_t word = 0x03020100u + (uint32_t)lane;
    const uint32_t wbase = (uint32_t)lane * (R * C * 4);
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        asm volatile("" : "+v"(word));
        static_for<0, 16>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            // left column of this step's tile: lane l-1's right column of the last step
            int32_t lf[R];
#pragma unroll
            for (int r = 0; r < R; ++r) lf[r] = __builtin_amdgcn_update_dpp(r + s, rc[r], 0x138, 0xF, 0xF, false);
            // scores: one v_perm per column gives 4 rows' bytes
            uint32_t sw[C][(R + 3) / 4];
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
                for (int q = 0; q < (R + 3) / 4; ++q) sw[c][q] = __builtin_amdgcn_perm(thi[c], tlo[c], word + q + s);
            int32_t x[R][C];
#pragma unroll
            for (int r = 0; r < R; ++r) {
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const int32_t diag = c == 0 ? (r == 0 ? dg : lf[r - 1]) : (r == 0 ? u[c - 1] : x[r - 1][c - 1]);
                    const int32_t up = r == 0 ? u[c] : x[r - 1][c];
                    const int32_t left = c == 0 ? lf[r] : x[r][c - 1];
                    const int32_t d = diag + (int32_t)(int8_t)(uint8_t)(sw[c][r >> 2] >> (8 * (r & 3)));
                    x[r][c] = max(max(d, up), left);
                }
            }
            dg = lf[R - 1];
#pragma unroll
            for (int c = 0; c < C; ++c) u[c] = x[R - 1][c];
#pragma unroll
            for (int r = 0; r < R; ++r) rc[r] = x[r][C - 1];
            // the tile to the ring, row-major within the lane's record
            char *p = ring + (s & 15) * kSlot + wbase;
            if constexpr (R * C == 1) {
                *(int32_t *)p = x[0][0];
            } else if constexpr (R * C == 2) {
                *(int2 *)p = make_int2(x[0][0], R == 2 ? x[1][0] : x[0][1]);
            } else {
#pragma unroll
                for (int q = 0; q < R * C / 4; ++q) {
                    const int e = 4 * q;
                    *(int4 *)(p + 16 * q) = make_int4(x[(e) / C][(e) % C], x[(e + 1) / C][(e + 1) % C],
                                                      x[(e + 2) / C][(e + 2) % C], x[(e + 3) / C][(e + 3) % C]);
                }
            }
        });
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    int32_t acc = dg;
#pragma unroll
    for (int c = 0; c < C; ++c) acc += u[c];
    acc += *(int32_t *)(ring + lane * 4);
    out[blockIdx.x * 64 + lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = c1 - c0;
}

template <int R, int C>
void run(int32_t *out, uint64_t *cyc, int grid, int iters) {
    hipLaunchKernelGGL((steps<R, C>), dim3(grid), dim3(64), 0, 0, 1, out, cyc);
    hipDeviceSynchronize();
    hipLaunchKernelGGL((steps<R, C>), dim3(grid), dim3(64), 0, 0, iters, out, cyc);
    hipDeviceSynchronize();
    uint64_t c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double st = 16.0 * iters;
    printf("R=%d C=%d grid %5d: %6.1f clk/step  %6.1f clk/row  %6.2f clk/cell-per-lane\n", R, C, grid, c / st,
           c / st / R, c / st / (R * C));
}

int main() {
    int32_t *out;
    uint64_t *cyc;
    hipMalloc(&out, 2048 * 64 * 4);
    hipMalloc(&cyc, 2048 * 8);
    const int iters = 20000;
    for (int grid : {256, 1024}) {
        run<1, 1>(out, cyc, grid, iters);
        run<1, 2>(out, cyc, grid, iters);
        run<1, 4>(out, cyc, grid, iters);
        run<2, 1>(out, cyc, grid, iters);
        run<4, 1>(out, cyc, grid, iters);
        run<8, 1>(out, cyc, grid, iters);
        run<2, 2>(out, cyc, grid, iters);
        run<4, 2>(out, cyc, grid, iters);
        run<8, 2>(out, cyc, grid, iters);
    }
    return 0;
}
