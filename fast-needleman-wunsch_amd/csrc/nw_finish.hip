// nw_finish.hip -- row-scan finisher for the leftover rows of a row band swept
// in horizontal strips (nw_fill_tband_async).
//
// The horizontal sweep cuts a band's R rows into strips of 256 rows that run
// side by side along all n1 columns.  The mpi-horz partition
// (src/mpi/mpi-horz-driver.cpp:31-32) gives every band after the first one row
// more than a multiple of 256 (its halo row) and the last band the remainder, so
// the band's last strip often holds a handful of rows -- and when the strips
// already fill the resident workers, that strip runs ALONE as a second pass over
// all n1 columns (config 4's last band: 65537 rows = 257 strips on 256 CUs, a
// full second sweep).  This kernel computes those rows instead, one row at a
// time across the whole width:
//
//   in the w form (w = t - GAP (i + j), row i global), the reference recurrence
//   (src/serial/serial.cpp:21-33) is
//     b_j = max(w[i-1][j-1] + s(j) - 2 GAP, w[i-1][j])       (reads row i-1 only)
//     w[i][j] = max(b_j, w[i][j-1]),   w[i][0] = 0            (a prefix maximum)
//   so a row is a prefix-max scan of b seeded with 0 -- exact for any GAP sign.
//
// Decomposition: the columns 1..n1 are cut into chunks of 256 * K; one
// workgroup (4 waves, K consecutive columns per thread) owns a chunk for all
// the rows.  Per row: each thread forms its b's and their running maximum
// (K v_max), the workgroup scans the thread totals (wave scan + 4 wave totals
// in LDS), the chunk's maximum is published as a look-back granule
// {tag: aggregate, value}, wave 0 looks back over its predecessors' granules
// (64 at a time, stopping at the nearest one that already carries its
// INCLUSIVE prefix) and publishes its own inclusive prefix: the decoupled
// look-back scan, one pass per row.  w is non-decreasing along a row, so the
// chunk's exclusive prefix IS w at the column left of it: the next row needs
// no value from any other workgroup.  Chunks are claimed from a ticket (ctrl[6])
// so every predecessor of a running chunk has started: no deadlock for any
// residency.  Each row is written back as 32 contiguous bytes per thread;
// the band's last row is also published into the next band's feed (w form,
// one granule per column) when the band has a consumer.
//
// Waits are bounded by the launch's watchdog (code 1, a granule wait, site 30) and
// abandoned at once when the error word is set -- e.g. by the fill before it, in
// which case nothing is computed or published.  The band's last row is published
// only if the error word is still clear when its row is done (wave 0 re-reads it),
// so no feed goes out after another chunk has given up.
#include <hip/hip_runtime.h>

#include "nw_dev.h"
#include "nw_internal.h"

namespace nw {

namespace {

constexpr int kFinThreads = 256;

__device__ __forceinline__ int32_t wave_max(int32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
    return v;
}

// Exclusive-prefix of chunk `k` for row slot `look` (k >= 1), by wave 0 of the
// workgroup: maximum over the predecessors' values back to the nearest one that
// carries its inclusive prefix (chunk -1 counts as inclusive with w[i][0] = 0).
// Returns kDead when it gave up.
__device__ __noinline__ int32_t look_back(const uint64_t *look, int32_t k, uint32_t tag_agg, uint32_t tag_inc,
                                          uint32_t *ctrl, uint64_t tmo) {
    const int lane = threadIdx.x & 63;
    int32_t carry = kNeg;
    int32_t j = k - 1;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t n = 1;; ++n) {
        const int32_t idx = j - lane;
        const uint64_t g = idx >= 0 ? gran_load(look + idx) : ((uint64_t)tag_inc << 32);
        const uint32_t tg = (uint32_t)(g >> 32);
        const uint64_t inc = __ballot(tg == tag_inc);
        const uint64_t ok = __ballot(tg == tag_inc || tg == tag_agg);
        const int lim = inc ? __builtin_ctzll(inc) : 63;
        const uint64_t need = lim == 63 ? ~0ull : ((2ull << lim) - 1ull);
        if ((ok & need) == need) {
            carry = max(carry, wave_max(lane <= lim ? (int32_t)(uint32_t)g : kNeg));
            if (inc) return carry;
            j -= 64;
            continue;
        }
        __builtin_amdgcn_s_sleep(1);
        if (n % kPollCheck == 0u) {  // (the error word: not a hot line, nw_dev.h wait_chunk)
            if (ctrl_load(ctrl + 1) != 0u) return kDead;
            if (__builtin_amdgcn_s_memrealtime() - t0 > tmo) {
                give_up(ctrl, 1u, 30, look + max(j, 0), tag_agg, (int64_t)j);
                return kDead;
            }
        }
    }
}

template <int K>
__global__ __launch_bounds__(kFinThreads) void nw_finish_rows(FinishArgs A) {
    __shared__ int32_t sh_chunk, sh_carry, sh_dead;
    __shared__ int32_t wtot[2][4];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) {
        sh_chunk = (int32_t)atomicAdd(A.ctrl + 6, 1u);
        sh_dead = ctrl_load(A.ctrl + 1) != 0u;  // the fill before gave up: leave everything
    }
    __syncthreads();
    if (sh_dead) return;
    const int32_t chunk = sh_chunk;
    const int64_t c0 = 1 + (int64_t)chunk * (kFinThreads * K) + (int64_t)tid * K;  // first column
    const int32_t g2 = 2 * A.gap;
    uint32_t a[K];
#pragma unroll
    for (int q = 0; q < K; ++q) a[q] = c0 + q <= A.n1 ? (uint32_t)A.s1[c0 + q - 1] : 0u;
    // the row above the first one (written by the fill), in the w form
    int32_t wp[K], wl;
    {
        const int64_t gi = A.grow0 + A.li0 - 1;
        const int32_t *prev = A.table + (A.li0 - 1) * A.pitch;
#pragma unroll
        for (int q = 0; q < K; ++q)
            wp[q] = c0 + q <= A.n1 ? (int32_t)(prev[c0 + q] - A.gap * (gi + c0 + q)) : kNeg;
        wl = c0 - 1 <= A.n1 ? (int32_t)(prev[c0 - 1] - A.gap * (gi + c0 - 1)) : kNeg;
    }
    for (int64_t r = 0; r < A.nrows; ++r) {
        const int64_t li = A.li0 + r, gi = A.grow0 + li;
        const uint32_t b = (uint32_t)A.s2[li - 1];
        int32_t lp[K];
        int32_t run = kNeg, d = wl;
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const int32_t s = (a[q] == b ? A.match : A.mismatch) - g2;
            run = max(run, max(d + s, wp[q]));
            d = wp[q];
            lp[q] = run;
        }
        // inclusive wave scan of the thread totals, then the 4 wave totals
        int32_t tot = run;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int32_t t = __shfl_up(tot, off, 64);
            if (lane >= off) tot = max(tot, t);
        }
        if (lane == 63) wtot[r & 1][wv] = tot;
        int32_t ex = __shfl_up(tot, 1, 64);
        if (lane == 0) ex = kNeg;
        __syncthreads();
        int32_t agg = kNeg, exw = kNeg;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            agg = max(agg, wtot[r & 1][w]);
            if (w < wv) exw = max(exw, wtot[r & 1][w]);
        }
        ex = max(ex, exw);
        if (wv == 0) {
            const uint32_t tag_agg = A.tag0 + 2u * (uint32_t)r, tag_inc = tag_agg + 1u;
            uint64_t *look = A.look + r * (int64_t)A.nchunks;
            int32_t carry = 0;
            if (chunk > 0) {
                if (lane == 0)
                    gran_store(look + chunk, ((uint64_t)tag_agg << 32) | (uint32_t)agg);
                carry = look_back(look, chunk, tag_agg, tag_inc, A.ctrl, A.timeout_ticks);
            }
            // the last row of a band with a consumer: publish it only while no chunk
            // has given up (chunk 0 never looks back, and a look-back can end before
            // another chunk's watchdog fires)
            if (A.feed_out != nullptr && r == A.nrows - 1 && carry != kDead && ctrl_load(A.ctrl + 1) != 0u)
                carry = kDead;
            if (lane == 0) {
                if (carry != kDead)
                    gran_store(look + chunk, ((uint64_t)tag_inc << 32) | (uint32_t)max(carry, agg));
                sh_carry = carry;
            }
        }
        __syncthreads();
        const int32_t carry = sh_carry;
        if (carry == kDead) return;  // (uniform: every thread read the same word)
        const int32_t pre = max(carry, ex);  // w[i][c0 - 1]
        int32_t w[K];
#pragma unroll
        for (int q = 0; q < K; ++q) w[q] = max(pre, lp[q]);
        int32_t *row = A.table + li * A.pitch;
        if (c0 + K - 1 <= A.n1) {
            typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int h = 0; h < K / 4; ++h) {
                i32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = w[4 * h + e] + (int32_t)(A.gap * (gi + c0 + 4 * h + e));
                *(i32x4 *)(row + c0 + 4 * h) = v;
            }
        } else {
#pragma unroll
            for (int q = 0; q < K; ++q)
                if (c0 + q <= A.n1) row[c0 + q] = w[q] + (int32_t)(A.gap * (gi + c0 + q));
        }
        if (A.feed_out != nullptr && r == A.nrows - 1) {  // the band's last row -> the next band
#pragma unroll
            for (int q = 0; q < K; ++q)
                if (c0 + q <= A.n1)
                    gran_store(A.feed_out + c0 + q, ((uint64_t)A.feed_tag << 32) | (uint32_t)w[q]);
            if (chunk == 0 && tid == 0) gran_store(A.feed_out, (uint64_t)A.feed_tag << 32);  // w[i][0] = 0
            // the padding up to the feed's 64-granule blocks: the consumer takes granules
            // 16 at a time (values beyond n1 are never stored)
            if (chunk == A.nchunks - 1)
                for (int64_t c = A.n1 + 1 + tid; c < (A.n1 + 64) / 64 * 64; c += kFinThreads)
                    gran_store(A.feed_out + c, (uint64_t)A.feed_tag << 32);
        }
        wl = pre;
#pragma unroll
        for (int q = 0; q < K; ++q) wp[q] = w[q];
    }
}

}  // namespace

int finish_chunk_cols(int64_t n1, int cus) {
    return (n1 + kFinThreads * 8 - 1) / (kFinThreads * 8) <= 8 * (int64_t)cus ? kFinThreads * 8 : kFinThreads * 32;
}

int launch_finish_rows(const FinishArgs &a, void *stream) {
    const int cols = a.chunk_cols;
    if (cols == kFinThreads * 8)
        hipLaunchKernelGGL(nw_finish_rows<8>, dim3((unsigned)a.nchunks), dim3(kFinThreads), 0, (hipStream_t)stream, a);
    else if (cols == kFinThreads * 32)
        hipLaunchKernelGGL(nw_finish_rows<32>, dim3((unsigned)a.nchunks), dim3(kFinThreads), 0, (hipStream_t)stream, a);
    else
        return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
}

}  // namespace nw
