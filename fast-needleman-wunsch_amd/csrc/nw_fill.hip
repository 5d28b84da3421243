// nw_fill.hip -- gfx950 (MI355X) Needleman-Wunsch scoring-table fill.
//
// Replaces the fill loops of the reference plugins
//   src/serial/serial.cpp:21-33, src/sentinel/sentinel-mt.cpp:40-62,
//   src/idxarray/idxarray-mt.cpp:43-66
// which all compute, row-major over an int32 table of (n2+1) x (n1+1):
//   t[i][j] = max(t[i-1][j-1] + s(s1[j-1], s2[i-1]), t[i-1][j] + GAP, t[i][j-1] + GAP)
//   t[0][j] = j*GAP, t[i][0] = i*GAP                              (serial.cpp:16-17)
//
// Decomposition:
//   * The table is cut into vertical STRIPS of 64 columns.  One wave64 owns a
//     strip: lane l owns column c = 64p + l and sweeps the rows.  At step s lane l
//     computes row i = s - l (anti-diagonal wavefront inside the wave).
//       up   = t[i-1][c]   : the lane's own previous result (register)
//       left = t[i][c-1]   : lane l-1's previous result, moved by DPP wave_shr:1
//       diag = t[i-1][c-1] : lane l-1's result two steps back = last step's `left`
//     Lane 0 takes left/diag from the strip to its left (the "feed").
//   * Every value is written to a 128-row LDS ring (row-indexed); at the end of
//     each 64-step iteration the 64 rows that became complete are flushed as
//     row-contiguous 256-B segments (ds_read_b128 -> global_store_dwordx4).
//   * Strip-to-strip hand-off: the right column of strip p (lane 63) is
//     published per 64-row block as 8-byte {tag, value} granules written with
//     agent-scope atomic stores (the data is the flag; no fences).  Strip p+1
//     polls them with agent-scope loads.  This is the GPU analogue of
//     idxarray-mt's per-row progress counters (idxarray-mt.cpp:8,44,50-56).
//   * Strips are claimed from an atomic ticket in increasing order by a
//     persistent grid of single-wave workgroups, so a strip's producer is always
//     already running: deadlock-free for any grid size / residency.
//   * Pure int32 VALU + LDS + HBM stores; no MFMA (there is no contraction).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "nw_internal.h"

namespace nw {

// s_memrealtime runs at 100 MHz on gfx9: 20 s watchdog for every bounded spin.
constexpr uint64_t kTimeoutTicks = 100000000ull * 20ull;
constexpr int kLdsTile = kRing * kWave;          // int32 words of the staging ring
constexpr int kLdsWords = kLdsTile + kRing;      // + feed ring (left boundary)

__device__ __forceinline__ uint64_t gran_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gran_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ctrl_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Slow path of the hand-off: re-poll until every lane's granule carries `tag`
// (s_sleep between polls).  Bounded: gives up -- raising the error word -- after
// kTimeoutTicks, or at once if another wave already raised it.  Returns the last
// value read; the caller re-checks its tag.
__device__ __forceinline__ uint64_t wait_granules_slow(const uint64_t *g, uint32_t tag,
                                                    uint32_t *ctrl) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        __builtin_amdgcn_s_sleep(1);
        const uint64_t v = gran_load(g);
        if (__all((uint32_t)(v >> 32) == tag)) return v;
        if (ctrl_load(ctrl + 1) != 0u) return v;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) {
            if (threadIdx.x == 0) atomicCAS(ctrl + 1, 0u, 1u);
            return v;
        }
    }
}

// Row characters for the 64 steps of iteration `it`: pack g holds the bytes of
// rows 64*it + 4g - lane + {0,1,2,3} (one dword per 4 steps per lane).
__device__ __forceinline__ void load_packs(const uint32_t *__restrict__ q, int it, int lane,
                                           uint32_t (&pk)[16]) {
    const uint32_t *base = q + kQOff + (int64_t)it * 64 - lane;
#pragma unroll
    for (int g = 0; g < 16; ++g) pk[g] = base[4 * g];
}

// Compile-time loop: f(std::integral_constant<int, U>) for U in [B, E).
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// diag + s(a, b) for step u of a 4-step pack: byte (u & 3) of the row-character
// pack is compared with the lane's column character via an SDWA byte select
// (reference match test: raw byte equality, serial.cpp:23-24).  Kept as one asm
// statement per step so hipcc does not hoist 64 compares into SGPR masks.
//   UNIT (match - mismatch == 1, the reference default):  d = diag' + mm' + [a == b]
//   general:                                               d = diag' + (a == b ? ms' : mm')
// (diag' = diag + GAP is what the wave carries; ms' / mm' have GAP pre-subtracted.)
template <int BYTE, bool UNIT>
__device__ __forceinline__ int32_t diag_plus_sub(uint32_t pk, uint32_t a, int32_t tl_old,
                                                 int32_t msp, int32_t mmp) {
    int32_t d;
    if constexpr (UNIT) {
        asm volatile(
            "v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_%c4 src1_sel:DWORD\n\t"
            "v_addc_co_u32_e32 %0, vcc, %3, %5, vcc"
            : "=v"(d)
            : "v"(pk), "v"(a), "v"(tl_old), "i"(BYTE), "v"(mmp)
            : "vcc");
    } else {
        int32_t s;
        asm volatile(
            "v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_%c5 src1_sel:DWORD\n\t"
            "v_cndmask_b32_e32 %0, %3, %4, vcc"
            : "=v"(s)
            : "v"(pk), "v"(a), "v"(mmp), "v"(msp), "i"(BYTE)
            : "vcc");
        d = tl_old + s;
    }
    return d;
}

// 64 wavefront steps of one iteration (rows 64*it + u - lane, u = 0..63).
// RAMP: first iteration of a strip -- lanes whose row is still <= 0
// (lane >= u) keep their row-0 state and re-emit t[0][c].
template <bool RAMP, bool UNIT>
__device__ __forceinline__ void run_iter(int32_t *__restrict__ lds, int it, int lane,
                                         const uint32_t (&pk)[16], uint32_t a, int32_t msp,
                                         int32_t mmp, int32_t gap, int32_t &tg, int32_t &tl_old,
                                         uint32_t &laddr) {
    // feed (left strip's t[i][c0-1] + GAP for the 64 rows of this iteration),
    // read 4 rows per ds_read_b128, one group ahead of use.
    const int4 *feed4 = (const int4 *)(lds + kLdsTile + ((it & 1) << 6));
    int4 fq = feed4[0];
    int32_t rr = -lane - 1;  // RAMP: row index of this lane at the current step (opaque)
    static_for<0, 16>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        const int4 fcur = fq;
        if constexpr (g + 1 < 16) fq = feed4[g + 1];
        static_for<0, 4>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int u = 4 * g + k;
            const int32_t fv = k == 0 ? fcur.x : k == 1 ? fcur.y : k == 2 ? fcur.z : fcur.w;
            // left + GAP: lane l-1's last result; lane 0 gets the left strip's value.
            const int32_t tl_new = __builtin_amdgcn_update_dpp(fv, tg, 0x138 /*wave_shr:1*/,
                                                               0xF, 0xF, false);
            const int32_t d = diag_plus_sub<k, UNIT>(pk[g], a, tl_old, msp, mmp);
            int32_t t = max(max(d, tg), tl_new);  // max(diag+s, up+GAP, left+GAP)
            if constexpr (RAMP) {
                rr += 1;
                asm volatile("" : "+v"(rr));  // keep the per-step activity test in the loop
                const int32_t tgn = (rr >= 1) ? t + gap : tg;
                t = tgn - gap;
                tg = tgn;
            } else {
                tg = t + gap;
            }
            tl_old = tl_new;
            laddr = (laddr + 256u) & 0x7FFFu;  // ring row (i & 127) * 256 B + 4*lane
            *(int32_t *)((char *)lds + laddr) = t;
            (void)u;
        });
    });
}

// Flush block fb (64 rows that became complete) of strip p from the LDS ring to
// HBM as row-contiguous segments: each ds_read_b128 / global_store_dwordx4 pair
// moves 4 rows x 256 B.  The device table holds round_up(nRows, 64) rows, so the
// rows past n2 of the last block land in padding and no store is masked.  Then
// publish the strip's right column (lane 63's values) for rows of this block as
// {tag, value} granules for strip p+1 (the last strip publishes into its own,
// never-read slot: keeps the store count branch-free).
__device__ __forceinline__ void flush_block(const int32_t *__restrict__ lds, int fb, int lane,
                                            int32_t *dst, int64_t pitch, uint64_t *gout,
                                            uint32_t tag_out) {
    const int sbase = (fb & 1) << 6;
    const int rsub = lane >> 4, csub = (lane & 15) * 4;
    int32_t *g = dst + rsub * pitch + csub;
    const int4 *src = (const int4 *)(lds + (sbase + rsub) * 64 + csub);
    const int64_t step4 = 4 * pitch;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int4 v = src[q * 64];  // 4 rows down = 4*64 words = 64 int4
        *(int4 *)(g + q * step4) = v;
    }
    const int32_t v = lds[(sbase + lane) * 64 + 63];
    gran_store(gout + lane, ((uint64_t)tag_out << 32) | (uint32_t)v);
}

template <bool UNIT>
__device__ void process_strip(const FillArgs &A, int32_t *__restrict__ lds, int p, int lane) {
    const int64_t c = (int64_t)p * 64 + lane;
    const int32_t gap = A.gap;
    const int32_t msp = A.match - gap, mmp = A.mismatch - gap;
    const uint32_t a = (c >= 1 && c <= A.n1) ? (uint32_t)A.s1[c - 1] : 0u;
    int32_t top = (int32_t)(c * (int64_t)gap);
    if (A.top != nullptr && c <= A.n1) top = A.top[c];
    int32_t tg = top + gap;  // t[0][c] + GAP
    int32_t tl_old = 0;
    uint32_t laddr = ((uint32_t)(-1 - lane) & 127u) * 256u + (uint32_t)lane * 4u;

    const bool has_left = p > 0;
    const uint64_t *gin = A.gran + (int64_t)((p + A.M - 1) % A.M) * A.gstride + lane;
    uint64_t *gout = A.gran + (int64_t)(p % A.M) * A.gstride;
    const uint32_t tag_in = A.tagbase + (uint32_t)p;
    const uint32_t tag_out = A.tagbase + (uint32_t)p + 1u;

    // Prefetch pipeline (all loads unconditional, so no loop-carried register
    // copies force an early s_waitcnt that would drain the flush stores):
    //   granules of block it+1 and row packs of iteration it+1 are issued at the
    //   start of iteration it, before that iteration's flush stores.
    const int lastb = A.nblocks - 1;
    uint64_t gv = gran_load(gin);  // block 0 (slot of strip p-1; unused when p == 0)
    uint32_t pkA[16], pkB[16];
    load_packs(A.rowpack, 0, lane, pkA);

    // One iteration: feed for block it, prefetch it+1, 64 steps, flush block it-1.
    // A watchdog trip only marks the strip dead; the iteration still issues the
    // same VMEM operations so every path into the next iteration is identical for
    // hipcc's s_waitcnt accounting, and the strip is abandoned at the boundary.
    bool dead = false;
    uint32_t nslow = 0;
    uint64_t wticks = 0;
    const uint64_t tstart = __builtin_amdgcn_s_memrealtime();
    auto iter = [&](int it, const uint32_t(&pk)[16], uint32_t(&pkn)[16], auto ramp) {
        constexpr bool RAMP = decltype(ramp)::value;  // first iteration: no block to flush yet
        if (it < A.nblocks) {
            int32_t fvv = kNeg;
            if (has_left) {
                if (!__all((uint32_t)(gv >> 32) == tag_in)) {
                    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
                    gv = wait_granules_slow(gin + (int64_t)it * 64, tag_in, A.ctrl);
                    dead = !__all((uint32_t)(gv >> 32) == tag_in);
                    nslow += 1;
                    wticks += __builtin_amdgcn_s_memrealtime() - w0;
                }
                fvv = (int32_t)(uint32_t)gv + gap;
            }
            lds[kLdsTile + ((it & 1) << 6) + lane] = fvv;
        }
        gv = gran_load(gin + (int64_t)min(it + 1, lastb) * 64);
        load_packs(A.rowpack, it + 1, lane, pkn);
        run_iter<RAMP, UNIT>(lds, it, lane, pk, a, msp, mmp, gap, tg, tl_old, laddr);
        if constexpr (!RAMP) {
            const int64_t row0 = (int64_t)(it - 1) * 64;
            int32_t *dst = A.table + row0 * A.pitch + (int64_t)p * 64;
            int64_t pitch = A.pitch;
            if (A.flags & 1) {  // debug timing mode: keep the stores, drop the HBM traffic
                dst = A.scratch + (int64_t)blockIdx.x * kScratchWords;
                pitch = kWave;
            }
            flush_block(lds, it - 1, lane, dst, pitch, gout + row0, tag_out);
        } else {
            // Nothing is complete yet.  Issue the same 17 stores into this
            // workgroup's scratch tile so that every path into the steady-state
            // loop carries the same VMEM count (hipcc's s_waitcnt bookkeeping then
            // never has to drain the previous flush to read the row packs).
            int32_t *scr = A.scratch + (int64_t)blockIdx.x * kScratchWords;
            flush_block(lds, 1, lane, scr, kWave, (uint64_t *)(scr + kWave * kWave), 0u);
        }
    };

    const int nit = A.nblocks + 1;  // iteration nblocks completes the last block
    iter(0, pkA, pkB, std::true_type{});
    for (int it = 1; it < nit && !dead; it += 2) {
        iter(it, pkB, pkA, std::false_type{});
        if (it + 1 >= nit || dead) break;
        iter(it + 1, pkA, pkB, std::false_type{});
    }
    if (A.trace != nullptr && lane == 0) {
        uint64_t *tr = A.trace + (int64_t)p * 4;
        tr[0] = tstart;
        tr[1] = __builtin_amdgcn_s_memrealtime();
        tr[2] = nslow;
        tr[3] = wticks;
    }
}

template <bool UNIT>
__global__ __launch_bounds__(64) void nw_fill_strips(FillArgs A) {
    __shared__ __attribute__((aligned(16))) int32_t lds[kLdsWords];
    const int lane = threadIdx.x;
    for (;;) {
        uint32_t p = 0;
        if (lane == 0) p = atomicAdd(A.ctrl, 1u);
        p = __builtin_amdgcn_readfirstlane(p);
        if (p >= (uint32_t)A.nstrips) break;
        process_strip<UNIT>(A, lds, (int)p, lane);
    }
}

// rowpack[idx] = B[x] | B[x+1] << 8 | B[x+2] << 16 | B[x+3] << 24, x = idx - kQOff,
// B[x] = s2[row0 + x - 1] for 1 <= x <= n2 (local rows of this launch), else 0.
__global__ void nw_rowpack(const uint8_t *__restrict__ s2, int64_t n2, int64_t row0,
                           uint32_t *__restrict__ q, int64_t qlen) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= qlen) return;
    const int64_t x = idx - kQOff;
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t y = x + k;
        const uint32_t b = (y >= 1 && y <= n2) ? (uint32_t)s2[row0 + y - 1] : 0u;
        v |= b << (8 * k);
    }
    q[idx] = v;
}

int64_t rowpack_len(int32_t nblocks) { return kQOff + 64 * ((int64_t)nblocks + 2) + 8; }

int launch_rowpack(const uint8_t *d_s2, int64_t n2, int64_t row0, uint32_t *d_q, int64_t qlen,
                   void *stream) {
    const int bs = 256;
    const int64_t nb = (qlen + bs - 1) / bs;
    hipLaunchKernelGGL(nw_rowpack, dim3((unsigned)nb), dim3(bs), 0, (hipStream_t)stream, d_s2,
                       n2, row0, d_q, qlen);
    return (int)hipGetLastError();
}

int launch_fill(const FillArgs &a, int grid, void *stream) {
    if (a.match - a.mismatch == 1)
        hipLaunchKernelGGL(nw_fill_strips<true>, dim3(grid), dim3(kWave), 0, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(nw_fill_strips<false>, dim3(grid), dim3(kWave), 0, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

const char *kernel_variant() { return "strip64-dpp-ldsring128-gran64"; }

}  // namespace nw
