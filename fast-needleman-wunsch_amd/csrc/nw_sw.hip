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

// First row-major cell holding the best value: workgroup y scans row blocks y,
// y + gridDim.x, ... of kLocRows rows in every strip / panel (any width: 256
// columns at a time) whose maximum is the best one -- a column's kLocRows loads
// are unconditional and independent, the first match is picked after -- and the
// workgroup and then the grid take the minimum key (row << 32 | column).
constexpr int kLocRows = 64;
constexpr int kLocMaxGrid = 4096;
__global__ __launch_bounds__(256) void nw_sw_locate(const int32_t *__restrict__ table, int64_t pitch,
                                                    int64_t n1, int64_t n2, int64_t col0, int32_t strip_cols,
                                                    const int32_t *__restrict__ smax, int32_t nstrips,
                                                    const int32_t *__restrict__ best,
                                                    uint64_t *__restrict__ key) {
    const int32_t b = *best;
    if (b <= 0) return;
    __shared__ unsigned long long kmin;
    if (threadIdx.x == 0) kmin = ~0ull;
    __syncthreads();
    const int64_t nblk = (n2 + kLocRows) / kLocRows;
    for (int64_t y = blockIdx.x; y < nblk; y += gridDim.x) {
        const int64_t r0 = y * kLocRows;
        const int nr = (int)min((int64_t)kLocRows, n2 + 1 - r0);
        for (int32_t p = 0; p < nstrips; ++p) {
            if (smax[p] != b) continue;
            for (int32_t x = threadIdx.x; x < strip_cols; x += 256) {
                const int64_t c = col0 + (int64_t)p * strip_cols + x;
                if (c > n1) break;
                const int32_t *col = table + r0 * pitch + c;
                int first = kLocRows;
#pragma unroll 16
                for (int rr = kLocRows - 1; rr >= 0; --rr) {
                    const int32_t v = rr < nr ? col[rr * pitch] : 0;
                    first = v == b ? rr : first;
                }
                if (first < kLocRows)
                    atomicMin(&kmin, ((unsigned long long)(r0 + first) << 32) | (unsigned long long)c);
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
    const int64_t grid = std::min<int64_t>((n2 + kLocRows) / kLocRows, kLocMaxGrid);
    hipLaunchKernelGGL(nw_sw_locate, dim3((unsigned)grid), dim3(256), 0, s, table, pitch, n1, n2, col0, strip_cols,
                       smax, nstrips, best, key);
    return (int)hipGetLastError();
}

// Half-word strip rings (nw_strips.h Lay::kHalf): a Smith-Waterman cell obeys
// 0 <= t <= M * min(i, j), M = max(match, mismatch) (t[i][0] = t[0][j] = 0 and
// each move adds at most M), so the rings' t mod 2^16 is exact wherever
// M * min(i, j) < 2^16.  The rest is the corner i, j >= K = ceil(2^16 / M) (one
// cell at 65536^2 with match 1): a wrong value there reaches only cells of the
// same corner (each cell's neighbours up/left/diag of a corner cell are in it or
// exact), and every value the strips produced there is <= the true one (max-plus
// with inputs <= the true ones, then the 0 floor and the wrap).  So the corner is
// recomputed here, in row-major order from its exact upper and left borders, and
// the strips' best-cell words raised to its true values; the host refuses the
// half-word shape when the corner exceeds kHalfFixMax cells.
__global__ __launch_bounds__(64) void nw_sw_fixup(int32_t *__restrict__ t, int64_t pitch,
                                                  const uint8_t *__restrict__ s1, const uint8_t *__restrict__ s2,
                                                  int32_t match, int32_t mismatch, int32_t gap, int64_t i0,
                                                  int64_t i1, int64_t j0, int64_t j1, int64_t col0, int32_t width,
                                                  int32_t *__restrict__ smax) {
    if (threadIdx.x != 0) return;
    for (int64_t i = i0; i <= i1; ++i) {
        int32_t left = t[i * pitch + j0 - 1];
        for (int64_t j = j0; j <= j1; ++j) {
            const int32_t d = t[(i - 1) * pitch + j - 1], u = t[(i - 1) * pitch + j];
            const int32_t sc = s1[j - 1] == s2[i - 1] ? match : mismatch;
            const int32_t v = max(max(0, d + sc), max(u + gap, left + gap));
            t[i * pitch + j] = v;
            left = v;
            atomicMax(smax + (j - col0) / width, v);
        }
    }
}

int64_t sw_half_corner(int32_t match, int32_t mismatch, int64_t n1, int64_t n2, int64_t *k) {
    const int64_t m = std::max(match, mismatch);
    if (m <= 0) {
        *k = INT64_MAX;
        return 0;
    }
    *k = (65536 + m - 1) / m;
    return std::max<int64_t>(0, n2 - *k + 1) * std::max<int64_t>(0, n1 - *k + 1);
}

int launch_sw_fixup(int32_t *table, int64_t pitch, int64_t n1, int64_t n2, const uint8_t *s1, const uint8_t *s2,
                    int32_t match, int32_t mismatch, int32_t gap, int64_t col0, int32_t strip_cols, int32_t *smax,
                    void *stream) {
    int64_t k = 0;
    if (sw_half_corner(match, mismatch, n1, n2, &k) == 0) return (int)hipSuccess;
    hipLaunchKernelGGL(nw_sw_fixup, dim3(1), dim3(64), 0, (hipStream_t)stream, table, pitch, s1, s2, match,
                       mismatch, gap, k, n2, k, n1, col0, strip_cols, smax);
    return (int)hipGetLastError();
}

// Traceback, parallel over windows.  The path from the best cell runs up and
// left through cells with t > 0, taking at every cell the first move that
// reproduces t (diag, then up, then left -- the order of serial.cpp:24-30's max).
// A ROUND from a start cell (is, js) cuts the rows above it into WINDOWS of kTbR
// rows, all skewed onto the diagonal through (is, js): window k's cell (r, x) is
// table cell (i0 + r, dj + r + x), i0 = is - (k+1) kTbR + 1, dj = js - is + i0 - B,
// x in [0, 2B], so a diagonal move keeps x, up is x + 1, left x - 1, and window
// k+1's bottom row continues window k's top row at the same x.
//   nw_tb_windows (one workgroup per window, all at once): the move code of every
//     cell (from the table, L2-resident neighbours), kept for nw_tb_emit, and for
//     every entry x of the bottom row the EXIT of the path from there: out of the
//     top at x' (continue in window k+1), a stop (t = 0, row / column 0: the
//     path's first cell), a move out of the band (the round restarts from that
//     cell, re-centred), or no matching move (not a Smith-Waterman table);
//   nw_tb_chain (one workgroup): follows the exits window to window from x = B --
//     one LDS read per window, exit tables staged kChain windows at a time --
//     giving each window its entry and its ops offset;
//   nw_tb_emit (one workgroup per window): walks its window from its entry and
//     writes the ops at its offset.
// A path that drifts more than B columns off the round's diagonal costs another
// round (re-centred at the cell where it left); run_sw_traceback loops rounds.
constexpr int kTbR = 64;                     // rows per window
constexpr int kTbBMax = 256;                 // band half-width B <= kTbBMax
constexpr int kTbWMax = 2 * kTbBMax + 1;     // cells per window row, W = 2B + 1
constexpr int kTbThreads = 512;
constexpr int kChain = 32;                   // windows per LDS chunk of nw_tb_chain
enum : uint8_t { kCStop = 0, kCDiag = 1, kCUp = 2, kCLeft = 3, kCBad = 4 };
enum : uint32_t { kXCont = 0, kXStop = 1, kXOut = 2, kXBad = 3 };
// exit record: kind 0-1 | moves 2-11 | row 12-18 | column 19-28 (kXCont: the
// column entered in the next window; otherwise the cell where the walk ended)
__device__ __forceinline__ uint32_t xrec(uint32_t kind, uint32_t cnt, uint32_t r, uint32_t x) {
    return kind | (cnt << 2) | (r << 12) | (x << 19);
}

// One window's walk from entry x (row kTbR - 1) over its move codes cd[]: calls
// emit(op) per move (0 diag, 1 up, 2 left); returns the exit record.
template <typename F>
__device__ __forceinline__ uint32_t tb_walk(const uint8_t *cd, int W, int x, F &&emit) {
    int r = kTbR - 1;
    uint32_t cnt = 0;
    for (;;) {
        const uint8_t c = cd[r * W + x];
        if (c == kCStop) return xrec(kXStop, cnt, r, x);
        if (c == kCBad) return xrec(kXBad, cnt, r, x);
        const int nx = c == kCUp ? x + 1 : c == kCLeft ? x - 1 : x;
        if (nx < 0 || nx >= W) return xrec(kXOut, cnt, r, x);  // (the move is the next round's)
        emit(c == kCDiag ? 0u : c == kCUp ? 1u : 2u);
        ++cnt;
        if (c != kCLeft && r == 0) return xrec(kXCont, cnt, 0, nx);
        r = c == kCLeft ? r : r - 1;
        x = nx;
    }
}

__global__ __launch_bounds__(kTbThreads) void nw_tb_windows(const int32_t *__restrict__ table, int64_t pitch,
                                                            int64_t n1, const uint8_t *__restrict__ s1,
                                                            const uint8_t *__restrict__ s2, int32_t match,
                                                            int32_t mismatch, int32_t gap, int64_t is, int64_t js,
                                                            int32_t B, uint8_t *__restrict__ codes,
                                                            uint32_t *__restrict__ exits) {
    __shared__ uint8_t cd[kTbR * kTbWMax];
    const int W = 2 * B + 1;
    const int k = blockIdx.x;
    const int64_t i0 = is - (int64_t)(k + 1) * kTbR + 1;
    const int64_t dj = js - is + i0 - B;
    const int ncell = kTbR * W;
    uint8_t *gcd = codes + (int64_t)k * ncell;
#pragma unroll 4
    for (int e = threadIdx.x; e < ncell; e += kTbThreads) {
        const int r = e / W, x = e - r * W;
        const int64_t i = i0 + r, j = dj + r + x;
        const bool in = i >= 1 && j >= 1 && j <= n1;
        // loads from clamped addresses (issued together), the decision after
        const int64_t ic = in ? i : 1, jc = in ? j : 1;
        const int32_t *row = table + ic * pitch;
        const int32_t t = row[jc], td = row[jc - 1 - pitch], tu = row[jc - pitch], tl = row[jc - 1];
        const int32_t sc = s1[jc - 1] == s2[ic - 1] ? match : mismatch;
        uint8_t c = kCStop;
        if (in && t > 0) c = t == td + sc ? kCDiag : t == tu + gap ? kCUp : t == tl + gap ? kCLeft : kCBad;
        cd[e] = c;
        gcd[e] = c;
    }
    __syncthreads();
    for (int x = threadIdx.x; x < W; x += kTbThreads) exits[(int64_t)k * W + x] = tb_walk(cd, W, x, [](uint32_t) {});
}

// ctl: [0] ops so far, [1] how the round ended (kXStop / kXCont|kXOut = restart /
// kXBad / 4 = ops buffer too small), [2..3] the begin cell or the restart cell,
// [4] windows holding ops this round.  wentry[k] = {entry x, ops offset}.
__global__ __launch_bounds__(1024) void nw_tb_chain(const uint32_t *__restrict__ exits, int32_t nwin, int32_t B,
                                                    int64_t is, int64_t js, int64_t ops_cap,
                                                    int64_t *__restrict__ wentry, int64_t *__restrict__ ctl) {
    __shared__ uint32_t ex[kChain * kTbWMax];
    __shared__ int64_t st[3];  // entry x, ops offset, done
    const int W = 2 * B + 1;
    const int tid = threadIdx.x;
    if (tid == 0) {
        st[0] = B;
        st[1] = ctl[0];
        st[2] = 0;
    }
    for (int k0 = 0; k0 < nwin; k0 += kChain) {
        const int nk = min(kChain, nwin - k0);
        for (int e = tid; e < nk * W; e += 1024) ex[e] = exits[(int64_t)k0 * W + e];
        __syncthreads();
        if (tid == 0) {
            int x = (int)st[0];
            int64_t off = st[1];
            for (int kk = 0; kk < nk; ++kk) {
                const int k = k0 + kk;
                wentry[2 * k] = x;
                wentry[2 * k + 1] = off;
                const uint32_t rec = ex[kk * W + x];
                const uint32_t kind = rec & 3u, cnt = (rec >> 2) & 1023u, r = (rec >> 12) & 127u, xx = rec >> 19;
                off += cnt;
                x = (int)xx;
                if (kind == kXCont && k + 1 < nwin) continue;
                // the round ends in window k
                const int64_t i0 = is - (int64_t)(k + 1) * kTbR + 1, dj = js - is + i0 - B;
                ctl[1] = off > ops_cap ? 4 : (int64_t)kind;
                ctl[2] = kind == kXCont ? i0 - 1 : i0 + r;
                ctl[3] = kind == kXCont ? dj - 1 + xx : dj + r + xx;
                ctl[4] = k + 1;
                ctl[0] = off;
                st[2] = 1;
                break;
            }
            st[0] = x;
            st[1] = off;
        }
        __syncthreads();
        if (st[2]) break;
    }
}

__global__ __launch_bounds__(256) void nw_tb_emit(const uint8_t *__restrict__ codes, int32_t B,
                                                  const int64_t *__restrict__ wentry, const int64_t *__restrict__ ctl,
                                                  uint8_t *__restrict__ ops) {
    __shared__ uint32_t cdw[kTbR * kTbWMax / 4 + 1];
    __shared__ uint8_t ob[2 * kTbR + kTbWMax + 8];
    __shared__ int32_t nop;
    const int k = blockIdx.x;
    if (k >= ctl[4] || ctl[1] == 4) return;
    const int W = 2 * B + 1, ncell = kTbR * W;  // (a multiple of 4: kTbR is)
    const uint32_t *g = (const uint32_t *)(codes + (int64_t)k * ncell);
    for (int e = threadIdx.x; e < ncell / 4; e += 256) cdw[e] = g[e];
    __syncthreads();
    if (threadIdx.x == 0) {
        int q = 0;
        tb_walk((const uint8_t *)cdw, W, (int)wentry[2 * k], [&](uint32_t op) { ob[q++] = (uint8_t)op; });
        nop = q;
    }
    __syncthreads();
    const int64_t off = wentry[2 * k + 1];
    for (int m = threadIdx.x; m < nop; m += 256) ops[off + m] = ob[m];
}

size_t sw_tb_scratch_bytes(int32_t maxwin, int32_t band) {
    const size_t W = 2 * (size_t)band + 1;
    return 64 + (size_t)maxwin * (16 + 4 * W + kTbR * W);
}

int run_sw_traceback(const int32_t *table, int64_t pitch, int64_t n1, const uint8_t *s1, const uint8_t *s2,
                     int32_t match, int32_t mismatch, int32_t gap, int64_t end_i, int64_t end_j, uint8_t *ops,
                     int64_t ops_cap, void *scratch, int32_t maxwin, int32_t band, int64_t *info, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    for (int q = 0; q < 10; ++q) info[q] = 0;
    if (band < 1 || band > kTbBMax || maxwin < 1) return (int)hipErrorInvalidValue;
    const int W = 2 * band + 1;
    int64_t *ctl = (int64_t *)scratch;
    int64_t *wentry = ctl + 8;
    uint32_t *exits = (uint32_t *)(wentry + 2 * (size_t)maxwin);
    uint8_t *codes = (uint8_t *)(exits + (size_t)maxwin * W);
    hipError_t e = hipMemsetAsync(ctl, 0, 64, s);
    if (e != hipSuccess) return (int)e;
    int64_t ci = end_i, cj = end_j, h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (;;) {
        if (ci <= 0 || cj <= 0) {  // row / column 0: the path's first cell
            info[1] = ci;
            info[2] = cj;
            break;
        }
        const int32_t nwin = (int32_t)std::min<int64_t>((ci + kTbR) / kTbR, maxwin);
        hipLaunchKernelGGL(nw_tb_windows, dim3((unsigned)nwin), dim3(kTbThreads), 0, s, table, pitch, n1, s1, s2,
                           match, mismatch, gap, ci, cj, band, codes, exits);
        hipLaunchKernelGGL(nw_tb_chain, dim3(1), dim3(1024), 0, s, exits, nwin, band, ci, cj, ops_cap, wentry, ctl);
        hipLaunchKernelGGL(nw_tb_emit, dim3((unsigned)nwin), dim3(256), 0, s, codes, band, wentry, ctl, ops);
        if ((e = hipGetLastError()) != hipSuccess) return (int)e;
        if ((e = hipMemcpyAsync(h, ctl, sizeof h, hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return (int)e;
        info[4] += 1;     // rounds
        info[5] += nwin;  // windows
        info[0] = h[0];
        if (h[1] == kXStop) {
            info[1] = h[2];
            info[2] = h[3];
            break;
        }
        if (h[1] == kXBad || h[1] == 4) {
            info[3] = h[1] == 4 ? 1 : 2;  // ops buffer too small / not a Smith-Waterman table
            info[1] = h[2];
            info[2] = h[3];
            break;
        }
        ci = h[2];  // kXCont past the round's last window, or kXOut: re-centre there
        cj = h[3];
    }
    return (int)hipSuccess;
}

}  // namespace nw
