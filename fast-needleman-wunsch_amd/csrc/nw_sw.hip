// nw_sw.hip -- Smith-Waterman best cell and on-device traceback (BASELINE config 5).
//
// The reference has no local alignment (its README only states the intent), so
// the conventions here are the build's own and the oracle is the CPU restatement
// oracle/nw_oracle.c (nw_oracle_sw_*), parity "unpinned" against the reference:
//   * table: t[i][0] = t[0][j] = 0, t[i][j] = max(0, t[i-1][j-1] + s(s1[j-1], s2[i-1]),
//     t[i-1][j] + GAP, t[i][j-1] + GAP)   (the fill kernel's SW modes, nw_fill.hip);
//   * best cell: the maximum, first in row-major order;
//   * traceback from it while t > 0, preferring diag > up > left -- the order in
//     which serial.cpp:24-30 takes its maximum (a, then b, then c).
// Both kernels are memory-latency work on a table already in HBM; neither is on
// the fill's store path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nw_internal.h"

namespace nw {

// best = max over the strips' words (one workgroup)
__global__ __launch_bounds__(256) void nw_sw_best(const int32_t *__restrict__ smax, int32_t nstrips,
                                                  int32_t *__restrict__ best, uint64_t *__restrict__ key) {
    __shared__ int32_t red[256];
    int32_t m = 0;
    for (int32_t p = threadIdx.x; p < nstrips; p += 256) m = max(m, smax[p]);
    red[threadIdx.x] = m;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        best[0] = red[0];
        *key = ~0ull;
    }
}

// First row-major cell holding the best value: workgroup (p, rb) scans strip p's
// columns over rows [rb*kLocRows, ...) if the strip's maximum is the best one;
// each thread keeps the first row of its column, the workgroup and then the grid
// take the minimum key (row << 32 | column).
constexpr int kLocRows = 512;
__global__ __launch_bounds__(256) void nw_sw_locate(const int32_t *__restrict__ table, int64_t pitch,
                                                    int64_t n1, int64_t n2, int64_t col0, int32_t strip_cols,
                                                    const int32_t *__restrict__ smax,
                                                    const int32_t *__restrict__ best,
                                                    uint64_t *__restrict__ key) {
    const int32_t p = blockIdx.x;
    const int32_t b = *best;
    if (b <= 0 || smax[p] != b) return;
    __shared__ unsigned long long kmin;
    if (threadIdx.x == 0) kmin = ~0ull;
    __syncthreads();
    const int64_t c = col0 + (int64_t)p * strip_cols + threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.y * kLocRows;
    const int64_t r1 = min(r0 + kLocRows, n2 + 1);
    if ((int)threadIdx.x < strip_cols && c <= n1) {
        for (int64_t r = r0; r < r1; ++r) {
            if (table[r * pitch + c] == b) {
                atomicMin(&kmin, ((unsigned long long)r << 32) | (unsigned long long)c);
                break;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && kmin != ~0ull) atomicMin((unsigned long long *)key, kmin);
}

int launch_sw_locate(const int32_t *table, int64_t pitch, int64_t n1, int64_t n2, int64_t col0,
                     int32_t strip_cols, const int32_t *smax, int32_t nstrips, uint64_t *key, int32_t *best,
                     void *stream) {
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(nw_sw_best, dim3(1), dim3(256), 0, s, smax, nstrips, best, key);
    const int64_t rb = (n2 + 1 + kLocRows - 1) / kLocRows;
    hipLaunchKernelGGL(nw_sw_locate, dim3((unsigned)nstrips, (unsigned)rb), dim3(256), 0, s, table, pitch, n1, n2,
                       col0, strip_cols, smax, best, key);
    return (int)hipGetLastError();
}

// Traceback: one workgroup of 1024 threads.  The table around the current cell
// is staged in LDS a window at a time -- rows [i0, i] x columns [j0, j], at most
// (kWin+1)^2 int32, every thread issuing all its loads before it waits -- with
// the window's characters; all threads then classify every cell of the window
// (the move the walk would take there: diag if t == t[i-1][j-1] + s, else up if
// t == t[i-1][j] + GAP, else left, or "stop" where t == 0), and thread 0 follows
// the codes -- one LDS byte per step -- writing one op per step, until it stops or
// reaches the window's top row / left column, where the next window is staged.
constexpr int kWin = 127;                       // (kWin+1)^2 int32 = 64 KB of LDS
constexpr int kTbThreads = 1024;
constexpr int kTbPer = ((kWin + 1) * (kWin + 1) + kTbThreads - 1) / kTbThreads;  // loads per thread
__global__ __launch_bounds__(kTbThreads) void nw_sw_traceback(
    const int32_t *__restrict__ table, int64_t pitch, const uint8_t *__restrict__ s1,
    const uint8_t *__restrict__ s2, int32_t match, int32_t mismatch, int32_t gap, int64_t end_i, int64_t end_j,
    uint8_t *__restrict__ ops, int64_t ops_cap, int64_t *__restrict__ info) {
    constexpr int W = kWin + 1;
    __shared__ int32_t win[W * W];
    __shared__ uint8_t code[W * W];
    __shared__ uint8_t c1[W], c2[W];
    __shared__ int64_t st[4];  // i, j, steps, status (done flag in the sign of i)
    const int tid = threadIdx.x;
    if (tid == 0) {
        st[0] = end_i;
        st[1] = end_j;
        st[2] = 0;
        st[3] = 0;
    }
    __syncthreads();
    for (;;) {
        const int64_t i = st[0], j = st[1];
        if (i <= 0 || j <= 0 || st[3] != 0) break;
        const int64_t i0 = i > kWin ? i - kWin : 0, j0 = j > kWin ? j - kWin : 0;
        const int rows = (int)(i - i0 + 1), cols = (int)(j - j0 + 1);
        int32_t v[kTbPer];
#pragma unroll
        for (int k = 0; k < kTbPer; ++k) {
            const int e = tid + k * kTbThreads, r = e / W, c = e % W;
            v[k] = (r < rows && c < cols) ? table[(i0 + r) * pitch + j0 + c] : 0;
        }
#pragma unroll
        for (int k = 0; k < kTbPer; ++k) {
            const int e = tid + k * kTbThreads;
            if (e < W * W) win[e] = v[k];
        }
        if (tid < W) {
            c1[tid] = (tid >= 1 && tid < cols) ? s1[j0 + tid - 1] : 0;  // column j0 + c holds s1[j0 + c - 1]
            c2[tid] = (tid >= 1 && tid < rows) ? s2[i0 + tid - 1] : 0;
        }
        __syncthreads();
        for (int e = tid; e < W * W; e += kTbThreads) {
            const int r = e / W, c = e % W;
            uint8_t cd = 3;
            if (r >= 1 && c >= 1 && r < rows && c < cols) {
                const int32_t t = win[e];
                if (t > 0) {
                    const int32_t sc = c1[c] == c2[r] ? match : mismatch;
                    cd = t == win[e - W - 1] + sc ? 0 : t == win[e - W] + gap ? 1 : t == win[e - 1] + gap ? 2 : 4;
                }
            }
            code[e] = cd;
        }
        __syncthreads();
        if (tid == 0) {
            int r = rows - 1, c = cols - 1;
            int64_t steps = st[2];
            bool done = false;
            while (r > 0 && c > 0) {
                const uint8_t cd = code[r * W + c];
                if (cd == 3) {
                    done = true;
                    break;
                }
                if (cd == 4) {
                    st[3] = 2;  // not a Smith-Waterman table
                    break;
                }
                if (steps >= ops_cap) {
                    st[3] = 1;
                    break;
                }
                ops[steps++] = cd;
                r -= cd != 2;
                c -= cd != 1;
            }
            if (!done && (i0 + r == 0 || j0 + c == 0)) done = true;  // row / column 0: t == 0
            st[0] = done ? -(i0 + r) - 1 : i0 + r;
            st[1] = j0 + c;
            st[2] = steps;
        }
        __syncthreads();
        if (st[0] < 0) break;
    }
    __syncthreads();
    if (tid == 0) {
        info[0] = st[2];
        info[1] = st[0] < 0 ? -st[0] - 1 : st[0];
        info[2] = st[1];
        info[3] = st[3];
    }
}

int launch_sw_traceback(const int32_t *table, int64_t pitch, const uint8_t *s1, const uint8_t *s2,
                        int32_t match, int32_t mismatch, int32_t gap, int64_t end_i, int64_t end_j,
                        uint8_t *ops, int64_t ops_cap, int64_t *info, void *stream) {
    hipLaunchKernelGGL(nw_sw_traceback, dim3(1), dim3(kTbThreads), 0, (hipStream_t)stream, table, pitch, s1, s2, match,
                       mismatch, gap, end_i, end_j, ops, ops_cap, info);
    return (int)hipGetLastError();
}

}  // namespace nw
