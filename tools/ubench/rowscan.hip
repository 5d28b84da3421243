// rowscan.hip -- cost of one ROW of the row-scan fill formulation, registers + LDS
// only (no global memory), on gfx950.
//
// Row-scan form (w = t - GAP*(i+j)): a wave owns 64*C consecutive columns of a
// row, lane l columns C*l .. C*l+C-1.  Row i from row i-1 (w):
//   d_k = w_{k-1} + s'_k            (w_{-1} = carry of the previous row)
//   p_k = max3(d_k, w_k, p_{k-1})   lane-local prefix max
//   S   = inclusive max-scan of p_{C-1} over the 64 lanes (6 DPP steps)
//   carry = max(S of lane l-1, L_i)  (L_i = left neighbour's last column)
//   w_k = max(p_k, carry)
// Reports shader cycles per row per wave for C = 1, 2, 4, 8 at W waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 rowscan.hip -o rowscan
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kNeg = -(1 << 29);

template <int CTRL, int RM>
__device__ __forceinline__ int32_t scan_step(int32_t x) {
    const int32_t t = __builtin_amdgcn_update_dpp(INT32_MIN, x, CTRL, RM, 0xF, false);
    return max(x, t);
}

__device__ __forceinline__ int32_t wave_scan_max(int32_t x) {
    x = scan_step<0x111, 0xF>(x);  // row_shr:1
    x = scan_step<0x112, 0xF>(x);  // row_shr:2
    x = scan_step<0x114, 0xF>(x);  // row_shr:4
    x = scan_step<0x118, 0xF>(x);  // row_shr:8
    x = scan_step<0x142, 0xA>(x);  // row_bcast:15
    x = scan_step<0x143, 0xC>(x);  // row_bcast:31
    return x;
}

template <int C, int TREE>
__global__ __launch_bounds__(1024) void rowscan(int rows, int32_t *out, unsigned long long *cyc, uint32_t sel0) {
    __shared__ __attribute__((aligned(16))) int32_t ring[16][4 * 512];  // per wave 4 rows x 64*C ints (C <= 8)
    __shared__ int32_t feed[16][64];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    feed[wv][lane] = lane * 3;
    __syncthreads();
    int32_t w[C];
    uint32_t tlo[C], thi[C];
#pragma unroll
    for (int k = 0; k < C; ++k) {
        w[k] = lane * C + k;
        tlo[k] = 0x03020302u + k;
        thi[k] = 0x02030203u;
    }
    int32_t cprev = lane * C - 1;
    int32_t *myring = &ring[wv][0];
    const int32_t *myfeed = &feed[wv][0];
    uint32_t sel = sel0 + (uint32_t)wv;
    int32_t Lq = myfeed[0];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < rows; r += 4) {
        uint32_t sc[C];
#pragma unroll
        for (int k = 0; k < C; ++k) sc[k] = __builtin_amdgcn_perm(thi[k], tlo[k], sel);
        int32_t Lnext = myfeed[(r + 4) & 63];  // prefetch next group's left values
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int32_t L = __builtin_amdgcn_readfirstlane(Lq) + q;
            int32_t d[C], p[C];
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const int32_t prev = k == 0 ? cprev : w[k - 1];
                d[k] = prev + (int32_t)(int8_t)(uint8_t)(sc[k] >> (8 * q));
            }
            int32_t tot;
            if constexpr (TREE) {
                // lane total by a tree (short critical path), prefixes off-path
                if constexpr (C == 1) {
                    tot = max(d[0], w[0]);
                    p[0] = tot;
                } else if constexpr (C == 2) {
                    tot = max(max(d[0], w[0]), max(d[1], w[1]));
                    p[0] = max(d[0], w[0]);
                    p[1] = tot;
                } else {
                    int32_t m[C];
#pragma unroll
                    for (int k = 0; k < C; ++k) m[k] = max(d[k], w[k]);
                    p[0] = m[0];
#pragma unroll
                    for (int k = 1; k < C; ++k) p[k] = max(p[k - 1], m[k]);
                    tot = p[C - 1];
                }
            } else {
                p[0] = max(d[0], w[0]);
#pragma unroll
                for (int k = 1; k < C; ++k) p[k] = max(max(d[k], w[k]), p[k - 1]);
                tot = p[C - 1];
            }
            const int32_t S = wave_scan_max(tot);
            int32_t carry = __builtin_amdgcn_update_dpp(L, S, 0x138 /*wave_shr:1*/, 0xF, 0xF, false);
            carry = max(carry, L);
#pragma unroll
            for (int k = 0; k < C; ++k) w[k] = max(p[k], carry);
            cprev = carry;
            // the row to the LDS ring (store waves would read it)
            int32_t *rp = myring + ((r + q) & 3) * 512 + lane * C;
            if constexpr (C == 1) {
                rp[0] = w[0];
            } else if constexpr (C == 2) {
                *(int2 *)rp = make_int2(w[0], w[1]);
            } else if constexpr (C == 4) {
                *(int4 *)rp = make_int4(w[0], w[1], w[2], w[3]);
            } else {
                *(int4 *)rp = make_int4(w[0], w[1], w[2], w[3]);
                *(int4 *)(rp + 4) = make_int4(w[4], w[5], w[6], w[7]);
            }
        }
        Lq = Lnext;
        sel = sel * 0x01000193u + 7u;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    int32_t acc = cprev;
#pragma unroll
    for (int k = 0; k < C; ++k) acc += w[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc + myring[lane];
    if (lane == 0) cyc[blockIdx.x * 16 + wv] = t1 - t0;
}

template <int C, int TREE>
static void run(int wps, int grid, int32_t *dout, unsigned long long *dcyc) {
    const int rows = 4096;
    const int threads = 64 * 4 * wps;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((rowscan<C, TREE>), dim3(grid), dim3(threads), 0, 0, rows, dout, dcyc, 0x00010203u);
        (void)hipDeviceSynchronize();
    }
    unsigned long long h[256 * 16];
    (void)hipMemcpy(h, dcyc, sizeof(h), hipMemcpyDeviceToHost);
    double s = 0;
    int n = 0;
    for (int b = 0; b < grid; ++b)
        for (int v = 0; v < 4 * wps; ++v) {
            s += (double)h[b * 16 + v];
            ++n;
        }
    const double cpr = s / n / rows;
    // cells per cycle per CU: 4*wps waves x 64*C cells per row
    printf("C=%d tree=%d waves/SIMD=%d grid=%d: %.1f cycles/row/wave  -> %.2f cells/cycle/CU\n", C, TREE, wps,
           grid, cpr, 4.0 * wps * 64 * C / cpr);
}

int main() {
    int32_t *dout;
    unsigned long long *dcyc;
    (void)hipMalloc(&dout, 256 * 1024 * 4);
    (void)hipMalloc(&dcyc, 256 * 16 * 8);
    for (int grid : {1, 256}) {
        for (int wps : {1, 2, 4}) {
            run<1, 0>(wps, grid, dout, dcyc);
            run<2, 0>(wps, grid, dout, dcyc);
            run<2, 1>(wps, grid, dout, dcyc);
            run<4, 0>(wps, grid, dout, dcyc);
            run<4, 1>(wps, grid, dout, dcyc);
            if (wps <= 2) run<8, 1>(wps, grid, dout, dcyc);
        }
    }
    return 0;
}
