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

#include <algorithm>

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

// First row-major cell holding the best value: workgroup (p, y) scans strip /
// panel p's columns (any width: 256 at a time) over the row blocks y, y +
// gridDim.y, ... of kLocRows rows if the strip's maximum is the best one; each
// thread keeps the first row of its column, the workgroup and then the grid take
// the minimum key (row << 32 | column).  gridDim.y is capped (the y dimension of
// a grid is limited), tall tables loop.
constexpr int kLocRows = 512;
constexpr int kLocMaxY = 4096;
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
    const int64_t nblk = (n2 + kLocRows) / kLocRows;
    for (int64_t y = blockIdx.y; y < nblk; y += gridDim.y) {
        const int64_t r0 = y * kLocRows;
        const int64_t r1 = min(r0 + kLocRows, n2 + 1);
        for (int32_t x = threadIdx.x; x < strip_cols; x += 256) {
            const int64_t c = col0 + (int64_t)p * strip_cols + x;
            if (c > n1) break;
            for (int64_t r = r0; r < r1; ++r) {
                if (table[r * pitch + c] == b) {
                    atomicMin(&kmin, ((unsigned long long)r << 32) | (unsigned long long)c);
                    break;
                }
            }
        }
        // a later row block cannot hold an earlier row: stop once one matched
        __syncthreads();
        if (kmin != ~0ull) break;
        __syncthreads();
    }
    if (threadIdx.x == 0 && kmin != ~0ull) atomicMin((unsigned long long *)key, kmin);
}

int launch_sw_locate(const int32_t *table, int64_t pitch, int64_t n1, int64_t n2, int64_t col0,
                     int32_t strip_cols, const int32_t *smax, int32_t nstrips, uint64_t *key, int32_t *best,
                     void *stream) {
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(nw_sw_best, dim3(1), dim3(256), 0, s, smax, nstrips, best, key);
    const int64_t rb = std::min<int64_t>((n2 + kLocRows) / kLocRows, kLocMaxY);
    hipLaunchKernelGGL(nw_sw_locate, dim3((unsigned)nstrips, (unsigned)rb), dim3(256), 0, s, table, pitch, n1, n2,
                       col0, strip_cols, smax, best, key);
    return (int)hipGetLastError();
}

// Traceback: one workgroup of 1024 threads.  The table around the current cell
// (i, j) is staged in LDS a window at a time: a band of kBandW = 2B+1 cells around
// the diagonal through (i, j) (the "entry diagonal"), over up to kBandR rows --
// window cell (r, x) is table cell (i0 + r, j - (rows-1-r) + x - B).  A diagonal
// move keeps x, up moves to x + 1, left to x - 1, so the three moves are the LDS
// index steps W, W - 1 and 1.  Smith-Waterman paths are mostly diagonal, so a band
// covers ~kBandR moves per window where a square window of the same LDS covers ~W.
// Every thread issues all its loads before it waits; all threads then classify
// every cell of the window with the move the walk takes there, stored as its
// index step (diag if t == t[i-1][j-1] + s; else up if t == t[i-1][j] + GAP; else
// left if t == t[i][j-1] + GAP), or a stop code: t == 0 (or row / column 0 of the
// table), the window's top row or band side (the walk continues in the next
// window from there), or "no move matches" (not a Smith-Waterman table).
// Doubling passes turn the codes into 4-move codes and thread 0 follows them --
// per 4 moves one dependent LDS read, the ops into an LDS buffer -- and all
// threads copy the window's ops out together.
constexpr int kBandB = 32;
constexpr int kBandW = 2 * kBandB + 1;          // 65 cells per window row
constexpr int kBandR = 252;                     // rows per window: 252 * 65 <= 16384 cells
constexpr int kTbThreads = 1024;
constexpr int kTbCells = kBandR * kBandW;
constexpr int kTbPer = (kTbCells + kTbThreads - 1) / kTbThreads;  // cells per thread
constexpr int kTbPad = kTbPer * kTbThreads;  // LDS arrays padded: no bounds checks (rows >= kBandR there)
constexpr uint8_t kMvLeft = 1, kMvUp = kBandW - 1, kMvDiag = kBandW;  // index steps
constexpr uint8_t kStop = 0, kEdge = 200, kBad = 255;
__global__ __launch_bounds__(kTbThreads) void nw_sw_traceback(
    const int32_t *__restrict__ table, int64_t pitch, int64_t n1, const uint8_t *__restrict__ s1,
    const uint8_t *__restrict__ s2, int32_t match, int32_t mismatch, int32_t gap, int64_t end_i, int64_t end_j,
    uint8_t *__restrict__ ops, int64_t ops_cap, int64_t *__restrict__ info) {
    constexpr int W = kBandW, B = kBandB;
    __shared__ int32_t win[kTbPad];
    __shared__ uint8_t code[kTbPad];
    __shared__ uint16_t cc2[kTbPad];
    __shared__ uint16_t ob[kBandR / 2 + kBandW + 2];  // the window's moves, 4 per entry (2 bits each | count << 8)
    __shared__ uint8_t c1[kBandR + kBandW], c2[kBandR];
    __shared__ int64_t st[5];  // i, j, steps, status (done flag in the sign of i), moves this window
    const int tid = threadIdx.x;
    if (tid == 0) {
        st[0] = end_i;
        st[1] = end_j;
        st[2] = 0;
        st[3] = 0;
        st[4] = 0;
    }
    __syncthreads();
    uint64_t tl = 0, tc = 0, tw = 0, nwin = 0;  // (thread 0) ticks loading / classifying / walking
    uint64_t tc1 = 0, tc2 = 0;                  // (of tc: the 1-step codes, the 2-step codes)
    for (;;) {
        const int64_t i = st[0], j = st[1];
        if (i <= 0 || j <= 0 || st[3] != 0) break;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        ++nwin;
        const int rows = (int)(i + 1 < kBandR ? i + 1 : kBandR);
        const int64_t i0 = i - (rows - 1);
        const int64_t jb = j - (rows - 1) - B;  // table column of window cell (r, x) = jb + r + x
        // r + x ranges over [0, kBandR + kBandW): the table's columns 1 and n1 as
        // offsets from jb, clamped into that range (32-bit compares in the classify pass)
        const int lo1 = (int)std::min<int64_t>(std::max<int64_t>(1 - jb, -1), kBandR + kBandW);
        const int hi = (int)std::min<int64_t>(std::max<int64_t>(n1 - jb, -1), kBandR + kBandW);
        int32_t v[kTbPer];
#pragma unroll
        for (int k = 0; k < kTbPer; ++k) {
            const int e = tid + k * kTbThreads, r = e / W, x = e % W;
            const int64_t gj = jb + r + x;
            v[k] = (e < kTbCells && r < rows && gj >= 0 && gj <= n1) ? table[(i0 + r) * pitch + gj] : 0;
        }
#pragma unroll
        for (int k = 0; k < kTbPer; ++k) {
            const int e = tid + k * kTbThreads;
            if (e < kTbCells) win[e] = v[k];
        }
        if (tid < kBandR + kBandW) {  // c1[r + x] = s1 character of column jb + r + x
            const int64_t gj = jb + tid;
            c1[tid] = (gj >= 1 && gj <= n1) ? s1[gj - 1] : 0;
        }
        if (tid < kBandR) c2[tid] = (tid < rows && i0 + tid >= 1) ? s2[i0 + tid - 1] : 0;
        __syncthreads();
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        #pragma unroll
        for (int kk = 0; kk < kTbPer; ++kk) {
            const int e = tid + kk * kTbThreads;
            const int r = e / W, x = e - r * W, q = r + x;
            uint8_t cd = kStop;
            if (r >= rows || q < lo1 || q > hi || i0 + r == 0) {
                cd = kStop;  // (outside the table, or its row / column 0)
            } else if (r == 0 || x == 0 || x == W - 1) {
                cd = kEdge;  // a neighbour lies outside the window
            } else {
                const int32_t t = win[e];
                if (t > 0) {
                    const int32_t sc = c1[q] == c2[r] ? match : mismatch;
                    cd = t == win[e - W] + sc        ? kMvDiag
                         : t == win[e - W + 1] + gap ? kMvUp
                         : t == win[e - 1] + gap     ? kMvLeft
                                                     : kBad;
                }
            }
            code[e] = cd;
        }
        __syncthreads();
        const uint64_t t1b = __builtin_amdgcn_s_memrealtime();
        // Multi-step codes by doubling, so that the walk below takes 4 moves per
        // dependent LDS read: a k-step code holds the moves from a cell (2 bits
        // each: 0 diag, 1 up, 2 left), their count and their total index step.
        //   c2 (uint16): moves 0-3 | count 4-5 | step 6-14
        //   c4 (uint32, in win's place -- no longer needed): moves 0-7 | count 8-10 | step 16-31
        auto mv1 = [](uint8_t d) -> uint32_t { return d == kMvDiag ? 0u : d == kMvUp ? 1u : 2u; };
        auto is_mv = [](uint8_t d) { return d == kMvDiag || d == kMvUp || d == kMvLeft; };
        #pragma unroll
        for (int kk = 0; kk < kTbPer; ++kk) {
            const int e = tid + kk * kTbThreads;
            // branch-free (the loads of all 16 cells issue together): a non-move
            // reads its own code again
            const uint8_t a = code[e];
            const bool ma = is_mv(a);
            const uint8_t b = code[e - (ma ? a : 0)];
            const bool mb = ma && is_mv(b);
            const uint32_t one = mv1(a) | (1u << 4) | ((uint32_t)a << 6);
            const uint32_t two = mv1(a) | (mv1(b) << 2) | (2u << 4) | ((uint32_t)(a + b) << 6);
            cc2[e] = (uint16_t)(mb ? two : ma ? one : 0u);
        }
        __syncthreads();
        const uint64_t t1c = __builtin_amdgcn_s_memrealtime();
        uint32_t *c4 = (uint32_t *)win;
        #pragma unroll
        for (int kk = 0; kk < kTbPer; ++kk) {
            const int e = tid + kk * kTbThreads;
            const uint32_t a = cc2[e];
            const uint32_t na = (a >> 4) & 3u, da = a >> 6;
            const uint32_t b = cc2[e - (na == 2 ? (int)da : 0)];  // (branch-free, as above)
            const uint32_t nb = na == 2 ? (b >> 4) & 3u : 0u, db = na == 2 ? b >> 6 : 0u;
            c4[e] = (a & 15u) | ((na == 2 ? b & 15u : 0u) << 4) | ((na + nb) << 8) | ((da + db) << 16);
        }
        __syncthreads();
        const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
        if (tid == 0) {
            int idx = (rows - 1) * W + B;
            int k = 0, q = 0;
            for (;;) {
                const uint32_t w = c4[idx];
                const int n = (int)((w >> 8) & 7u);
                if (n == 0) break;
                ob[q++] = (uint16_t)(w & 0x7FFu);
                k += n;
                idx -= (int)(w >> 16);
                if (n < 4) break;
            }
            const uint8_t d = code[idx];  // where the walk stopped: kStop, kEdge or kBad
            const int r = idx / W, x = idx % W;
            const int64_t steps = st[2];
            if (d == kBad) {
                st[3] = 2;  // not a Smith-Waterman table
            } else if (steps + k > ops_cap) {
                st[3] = 1;
            } else {
                st[0] = d == kStop ? -(i0 + r) - 1 : i0 + r;  // (kEdge: next window from here)
                st[1] = jb + r + x;
            }
            st[4] = k;
        }
        __syncthreads();
        {
            const int k = (int)st[4];
            const int64_t steps = st[2];
            if (st[3] == 0)
                for (int e = tid; 4 * e < k; e += kTbThreads) {
                    const uint32_t w = ob[e];
                    const int n = (int)(w >> 8);
                    for (int m = 0; m < n; ++m) ops[steps + 4 * e + m] = (uint8_t)((w >> (2 * m)) & 3u);
                }
        }
        __syncthreads();
        if (tid == 0 && st[3] == 0) st[2] += st[4];
        __syncthreads();
        const uint64_t t3 = __builtin_amdgcn_s_memrealtime();
        tl += t1 - t0;
        tc += t2 - t1;
        tc1 += t1b - t1;
        tc2 += t1c - t1b;
        tw += t3 - t2;
        if (st[0] < 0) break;
    }
    __syncthreads();
    if (tid == 0) {
        info[0] = st[2];
        info[1] = st[0] < 0 ? -st[0] - 1 : st[0];
        info[2] = st[1];
        info[3] = st[3];
        info[4] = (int64_t)tl;  // (diagnostics: s_memrealtime ticks, 100 MHz)
        info[5] = (int64_t)tc;
        info[6] = (int64_t)tw;
        info[7] = (int64_t)nwin;
        info[8] = (int64_t)tc1;
        info[9] = (int64_t)tc2;
    }
}

int launch_sw_traceback(const int32_t *table, int64_t pitch, int64_t n1, const uint8_t *s1, const uint8_t *s2,
                        int32_t match, int32_t mismatch, int32_t gap, int64_t end_i, int64_t end_j,
                        uint8_t *ops, int64_t ops_cap, int64_t *info, void *stream) {
    hipLaunchKernelGGL(nw_sw_traceback, dim3(1), dim3(kTbThreads), 0, (hipStream_t)stream, table, pitch, n1, s1, s2, match,
                       mismatch, gap, end_i, end_j, ops, ops_cap, info);
    return (int)hipGetLastError();
}

}  // namespace nw
