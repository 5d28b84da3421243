// nw_fill.hip -- gfx950 (MI355X) Needleman-Wunsch scoring-table fill.
//
// Replaces the fill loops of the reference plugins
//   src/serial/serial.cpp:21-33, src/sentinel/sentinel-mt.cpp:40-62,
//   src/idxarray/idxarray-mt.cpp:43-66
// which all compute, row-major over an int32 table of (n2+1) x (n1+1):
//   t[i][j] = max(t[i-1][j-1] + s(s1[j-1], s2[i-1]), t[i-1][j] + GAP, t[i][j-1] + GAP)
//   t[0][j] = j*GAP, t[i][0] = i*GAP                              (serial.cpp:16-17)
//
// Decomposition (DESIGN.md has the full picture):
//   * The table is cut into vertical SUPER-STRIPS of K*64 columns, one wave64
//     each, made of K 64-column SUB-STRIPS.  In sub-strip k lane l owns column
//     c = 64*(K*p + k) + l and at step s computes row i = s - 64k - l: an
//     anti-diagonal wavefront inside the wave, sub-strip k trailing k-1 by 64
//     steps.
//       up   = t[i-1][c]   : the lane's own previous result (register)
//       left = t[i][c-1]   : lane l-1's previous result, DPP wave_shr:1
//       diag = t[i-1][c-1] : lane l-1's result two steps back = last step's `left`
//     Lane 0 of sub-strip k >= 1 takes left/diag from lane 63 of sub-strip k-1
//     (DPP wave_ror:1 of the previous step -- an in-register hand-off); lane 0
//     of sub-strip 0 takes them from the super-strip to the left (the "feed").
//     The K chains are independent within a step, so they interleave (ILP).
//   * Every value is written to a 128-row LDS ring per sub-strip (row-indexed);
//     at the end of each 64-step iteration the 64 rows that became complete are
//     flushed as row-contiguous 256-B segments (ds_read_b128 ->
//     global_store_dwordx4, 4 rows per instruction).
//   * Super-strip to super-strip hand-off: the right column (sub-strip K-1,
//     lane 63) is published per 64-row block as 8-byte {tag, value} granules
//     with agent-scope atomic stores (the data is the flag; no fences); the next
//     super-strip polls them with agent-scope loads -- the GPU analogue of
//     idxarray-mt's per-row progress counters (idxarray-mt.cpp:8,44,50-56).
//   * Super-strips are claimed from an atomic ticket in increasing order by a
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
constexpr int kRingWords = kRing * kWave;  // int32 words of one sub-strip's staging ring
constexpr int kRingBytes = kRingWords * 4;

// Optional cap on this wave's outstanding VMEM operations (stores, mostly),
// enforced after every flush group: a poll of the left neighbour's granules
// waits (vmcnt is in-order) for every older store of the wave, so the depth of
// the store queue is hand-off latency.  0 = no cap (hipcc's own waits only).
#ifndef NW_VMCAP
#define NW_VMCAP 0
#endif
// s_waitcnt immediate (gfx9): vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4]<<14
constexpr int vmcnt_imm(int n) { return (n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14); }

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

// Row characters for the 64 steps of local iteration j: pack g holds the bytes
// of rows 64*j + 4g - lane + {0,1,2,3} (one dword per 4 steps per lane).
__device__ __forceinline__ void load_packs(const uint32_t *__restrict__ q, int j, int lane,
                                           uint32_t (&pk)[16]) {
    const uint32_t *base = q + kQOff + (int64_t)max(j, 0) * 64 - lane;
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

// Per-lane state of one super-strip.
template <int K>
struct Lanes {
    uint32_t a[K];   // column character of this lane in sub-strip k
    int32_t tg[K];   // t(current row of the lane) + GAP  (up + GAP for the next step)
    int32_t tl[K];   // last step's left + GAP  (= diag' for this step)
    int32_t rr[K];   // RAMP: row index of the lane in sub-strip k at the current step
};

// Sub-strip modes in an iteration: IDLE (not started), RAMP (first iteration,
// lanes with row <= 0 hold row 0), RUN.
enum Mode { IDLE = 0, RAMP = 1, RUN = 2 };

template <int IT>
constexpr int prologue_mode(int k) {
    return IT - k < 0 ? IDLE : (IT - k == 0 ? RAMP : RUN);
}

// 64 wavefront steps of one iteration for all K sub-strips.  MODES packs the
// mode of sub-strip k in bits [2k, 2k+1].  Sub-strips are processed from K-1
// down to 0 inside a step so that sub-strip k reads sub-strip k-1's register
// state of the PREVIOUS step.
template <int K, bool UNIT, int MODES>
__device__ __forceinline__ void run_iter(int32_t *__restrict__ lds, int it,
                                         const uint32_t (&pk)[K][16], int32_t msp, int32_t mmp,
                                         int32_t gap, Lanes<K> &S, uint32_t laddr,
                                         char *const (&fdst)[K], const int64_t (&fstep)[K],
                                         const uint32_t (&foff)[K],
                                         int lane) {
    // Interleaved flush: the ring half this iteration overwrites holds the block
    // that completed in the previous iteration.  Before the 4 steps of group g
    // overwrite its rows 4g..4g+3, those rows are read (ds_read_b128, 4 rows x
    // 64 columns) and stored (global_store_dwordx4, 4 x 256 B row segments), so
    // the 16 stores of a block trickle out one per 4 steps instead of in a burst.
    //   Addressing: fdst[k] is the block's uniform base (SGPRs; column c0+64k of
    //   the block's first row), foff[k] this lane's 32-bit byte offset (row rsub,
    //   column csub), fstep[k] the uniform byte stride of a 4-row group, so each
    //   store is global_store_dwordx4 voff, data, s[base] with no VALU address
    //   math.  The LDS read of group g+1 is issued during group g (in-order LDS
    //   returns), so the store never waits on a just-issued ds_read.
    const int rsub = lane >> 4, csub = (lane & 15) * 4;
    const int fbase = (((it & 1) << 6) + rsub) * 64 + csub;
    // feed of sub-strip 0 (left super-strip's t[i][c0-1] + GAP for the 64 rows
    // of this iteration), read 4 rows per ds_read_b128, one group ahead.
    const int4 *feed4 = (const int4 *)(lds + K * kRingWords + ((it & 1) << 6));
    int4 fq = feed4[0];
    // keep the 64 per-step ring offsets in-loop (2 VALU/step shared by all K
    // sub-strips) instead of letting hipcc hoist 64 address VGPRs
    asm volatile("" : "+v"(laddr));
    int4 fv[K];
#pragma unroll
    for (int k = 0; k < K; ++k) fv[k] = *(const int4 *)(lds + k * kRingWords + fbase);
    static_for<0, 16>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        const int4 fcur = fq;
        if constexpr (g + 1 < 16) fq = feed4[g + 1];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int4 v = fv[k];
            if constexpr (g + 1 < 16) fv[k] = *(const int4 *)(lds + k * kRingWords + fbase + (g + 1) * 256);
            *(int4 *)(fdst[k] + g * fstep[k] + foff[k]) = v;
        }
        if constexpr (NW_VMCAP > 0) __builtin_amdgcn_s_waitcnt(vmcnt_imm(NW_VMCAP));
        static_for<0, 4>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            constexpr int u = 4 * g + q;
            const uint32_t off = (laddr + 256u * (uint32_t)(u + 1)) & 0x7FFFu;  // ring row (i & 127)
            static_for<0, K>([&](auto kk) {
                constexpr int k = K - 1 - decltype(kk)::value;  // K-1 .. 0
                constexpr int mode = (MODES >> (2 * k)) & 3;
                if constexpr (mode != IDLE) {
                    int32_t lf;  // lane-0 source of `left`
                    if constexpr (k == 0) {
                        lf = q == 0 ? fcur.x : q == 1 ? fcur.y : q == 2 ? fcur.z : fcur.w;
                    } else {
                        // lane 0 <- lane 63 of sub-strip k-1, previous step (wave_ror:1)
                        lf = __builtin_amdgcn_update_dpp(0, S.tg[k - 1], 0x13C, 0xF, 0xF, false);
                    }
                    const int32_t tl_new = __builtin_amdgcn_update_dpp(lf, S.tg[k], 0x138 /*wave_shr:1*/,
                                                                       0xF, 0xF, false);
                    const int32_t d = diag_plus_sub<q, UNIT>(pk[k][g], S.a[k], S.tl[k], msp, mmp);
                    int32_t t = max(max(d, S.tg[k]), tl_new);  // max(diag+s, up+GAP, left+GAP)
                    if constexpr (mode == RAMP) {
                        S.rr[k] += 1;
                        asm volatile("" : "+v"(S.rr[k]));  // keep the activity test in the loop
                        const int32_t tgn = (S.rr[k] >= 1) ? t + gap : S.tg[k];
                        t = tgn - gap;
                        S.tg[k] = tgn;
                    } else {
                        S.tg[k] = t + gap;
                    }
                    S.tl[k] = tl_new;
                    *(int32_t *)((char *)lds + k * kRingBytes + off) = t;
                }
            });
        });
    });
}

// Flush one 64-row block of one sub-strip from its LDS ring to `dst` (row-major,
// `pitch` int32) as row-contiguous segments: each ds_read_b128 /
// global_store_dwordx4 pair moves 4 rows x 256 B.  `sbase` = ring row of the
// block's first row (0 or 64).
__device__ __forceinline__ void flush_rows(const int32_t *__restrict__ ring, int sbase, int lane,
                                           int32_t *dst, int64_t pitch) {
    const int rsub = lane >> 4, csub = (lane & 15) * 4;
    int32_t *g = dst + rsub * pitch + csub;
    const int4 *src = (const int4 *)(ring + (sbase + rsub) * 64 + csub);
    const int64_t step4 = 4 * pitch;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int4 v = src[q * 64];  // 4 rows down = 4*64 words = 64 int4
        *(int4 *)(g + q * step4) = v;
    }
}

template <int K, bool UNIT>
__device__ void process_strip(const FillArgs &A, int32_t *__restrict__ lds, int p, int lane) {
    const int32_t gap = A.gap;
    const int32_t msp = A.match - gap, mmp = A.mismatch - gap;
    const int64_t c0 = (int64_t)p * (64 * K);
    bool dead = false;
    // Row 0: the boundary t[0][c] = c*GAP (serial.cpp:16), or -- for a row band
    // (mpi-horz.cpp:16-40) -- the previous band's last row, taken from its halo
    // granules once they carry this launch's tag (bounded wait).
    int32_t top[K];
#pragma unroll
    for (int k = 0; k < K; ++k) top[k] = (int32_t)((c0 + 64 * k + lane) * (int64_t)gap);
    if (A.halo_in != nullptr) {
        const uint64_t h0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            bool ok = true;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int64_t c = min(c0 + 64 * k + lane, A.n1);
                const uint64_t g = __hip_atomic_load(A.halo_in + c, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_SYSTEM);
                top[k] = (int32_t)(uint32_t)g;
                ok &= (uint32_t)(g >> 32) == A.halo_tag;
            }
            if (__all(ok)) break;
            if (ctrl_load(A.ctrl + 1) != 0u) { dead = true; break; }
            if (__builtin_amdgcn_s_memrealtime() - h0 > kTimeoutTicks) {
                if (lane == 0) atomicCAS(A.ctrl + 1, 0u, 2u);
                dead = true;
                break;
            }
            __builtin_amdgcn_s_sleep(4);
        }
    }
    Lanes<K> S;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int64_t c = c0 + 64 * k + lane;
        S.a[k] = (c >= 1 && c <= A.n1) ? (uint32_t)A.s1[c - 1] : 0u;
        S.tg[k] = top[k] + gap;  // t[0][c] + GAP
        S.tl[k] = 0;
        S.rr[k] = -lane - 1;
    }
    // ring byte offset of this lane before step 0 of an even iteration: ring row
    // (s - lane) & 127 at step s (every sub-strip: sub-strip k stores row i at
    // ring row (i + 64k) & 127), + 4 * lane
    const uint32_t lbase = ((uint32_t)(-1 - lane) & 127u) * 256u + (uint32_t)lane * 4u;

    const bool has_left = p > 0;
    const uint64_t *gin = A.gran + (int64_t)((p + A.M - 1) % A.M) * A.gstride + lane;
    uint64_t *gout = A.gran + (int64_t)(p % A.M) * A.gstride;
    const uint32_t tag_in = A.tagbase + (uint32_t)p;
    const uint32_t tag_out = A.tagbase + (uint32_t)p + 1u;
    const int lastb = A.nblocks - 1;
    int32_t *scr = A.scratch + (int64_t)blockIdx.x * kScratchWords;
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; ++k) valid[k] = c0 + 64 * k < A.pitch;

    // Prefetch pipeline (all loads unconditional, so no loop-carried register
    // copies force an early s_waitcnt that would drain the flush stores): the
    // granules and row packs used by later iterations are issued at the start of
    // iteration it, before that iteration's flush stores.
    // Prefetch pipeline.  Everything an iteration reads from global memory (the
    // left neighbour's granules for its feed, the row-character packs of its K
    // sub-strips) is loaded TWO iterations ahead into 3-deep register rings:
    // under full store traffic a load queues behind this CU's stores for longer
    // than an iteration, and vmcnt is in-order, so a load consumed one iteration
    // later would stall the wave every iteration.  Buffer = issue iteration mod 3;
    // iteration i consumes buffer (i+1) % 3 and refills buffer i % 3.  All loads
    // are unconditional (clamped indices) so every path carries the same VMEM
    // count for hipcc's s_waitcnt bookkeeping.
    uint64_t gb[3];
    uint32_t pkb[3][K][16];
    gb[1] = gran_load(gin);                                  // block 0, for iteration 0
    gb[2] = gran_load(gin + (int64_t)min(1, lastb) * 64);    // block 1, for iteration 1
    gb[0] = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        load_packs(A.rowpack, 0 - k, lane, pkb[1][k]);
        load_packs(A.rowpack, 1 - k, lane, pkb[2][k]);
    }

    uint32_t nslow = 0;
    uint64_t wticks = 0;
    const uint64_t tstart = __builtin_amdgcn_s_memrealtime();
    const uint64_t cstart = __builtin_amdgcn_s_memtime();
    uint64_t tq1 = 0, tmid = 0;  // trace: times iterations nblocks/4 and nblocks/2 started

    // One iteration: feed for block it, prefetch for it+2, flush (interleaved
    // with the steps), 64 steps.  A watchdog trip only marks the strip dead; the
    // iteration still issues the same VMEM operations, so every path into the next
    // iteration is identical for s_waitcnt accounting, and the strip is abandoned
    // at the boundary.
    auto iter = [&](int it, auto cons_c, auto iss_c, auto modes) {
        constexpr int CONS = decltype(cons_c)::value;  // (it + 1) % 3
        constexpr int ISS = decltype(iss_c)::value;    // it % 3
        constexpr int MODES = decltype(modes)::value;
        if (A.trace != nullptr) {
            if (it == A.nblocks / 4) tq1 = __builtin_amdgcn_s_memrealtime();
            if (it == A.nblocks / 2) tmid = __builtin_amdgcn_s_memrealtime();
        }
        if (it < A.nblocks) {
            int32_t fvv = kNeg;
            if (has_left) {
                uint64_t gv = gb[CONS];  // block it, loaded two iterations ago
                if (!__all((uint32_t)(gv >> 32) == tag_in)) {
                    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
                    gv = wait_granules_slow(gin + (int64_t)it * 64, tag_in, A.ctrl);
                    dead = !__all((uint32_t)(gv >> 32) == tag_in);
                    nslow += 1;
                    wticks += __builtin_amdgcn_s_memrealtime() - w0;
                }
                fvv = (int32_t)(uint32_t)gv + gap;
            }
            lds[K * kRingWords + ((it & 1) << 6) + lane] = fvv;
        }
        gb[ISS] = gran_load(gin + (int64_t)min(it + 2, lastb) * 64);
#pragma unroll
        for (int k = 0; k < K; ++k) load_packs(A.rowpack, it + 2 - k, lane, pkb[ISS][k]);
        // Flush what completed in the PREVIOUS iteration (sub-strip k: block
        // it-2-k), interleaved with this iteration's steps (see run_iter).  The
        // prefetch loads above are issued first: vmcnt is in-order, so a load
        // waited for later never queues behind these stores.  Blocks outside the
        // table (not yet started / past the end / columns past the pitch) go to
        // this workgroup's scratch tile, so every iteration issues the same
        // K*16 + 1 stores.
        char *fdst[K];
        int64_t fstep[K];
        uint32_t foff[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int b = it - 2 - k;
            const bool ok = valid[k] && b >= 0 && b < A.nblocks && !(A.flags & 1);
            fdst[k] = (char *)(ok ? A.table + (int64_t)b * 64 * A.pitch + c0 + 64 * k : scr);
            const int64_t fp = ok ? A.pitch : (int64_t)kWave;
            fstep[k] = 16 * fp;  // bytes of 4 rows
            foff[k] = (uint32_t)(((lane >> 4) * fp + (lane & 15) * 4) * 4);
        }
        {
            // right column of the super-strip (sub-strip K-1, lane 63) for block b,
            // read before this iteration's steps overwrite the ring half
            const int sbase = (it & 1) << 6;
            const int b = it - 1 - K;
            const int32_t v = lds[(K - 1) * kRingWords + (sbase + lane) * 64 + 63];
            const bool ok = b >= 0 && b < A.nblocks;
            uint64_t *gp = ok ? gout + (int64_t)b * 64 + lane
                              : (uint64_t *)(scr + kWave * kWave) + lane;
            gran_store(gp, ((uint64_t)tag_out << 32) | (uint32_t)v);
        }
        run_iter<K, UNIT, MODES>(lds, it, pkb[CONS], msp, mmp, gap, S,
                                 lbase + (uint32_t)(it & 1) * (64u * 256u), fdst, fstep, foff, lane);
    };

    // sub-strip K-1 completes the last block in iteration nblocks-1+K; it is
    // flushed at the start of the next one (whose 64 steps are wasted work)
    const int nit = A.nblocks + K + 1;
    // prologue iterations 0..K-1 (sub-strips start one after another)
    static_for<0, K>([&](auto itc) {
        constexpr int IT = decltype(itc)::value;
        constexpr int MODES = (prologue_mode<IT>(0) | (prologue_mode<IT>(1) << 2) |
                               (prologue_mode<IT>(2) << 4) | (prologue_mode<IT>(3) << 6)) &
                              ((1 << (2 * K)) - 1);
        iter(IT, std::integral_constant<int, (IT + 1) % 3>{}, std::integral_constant<int, IT % 3>{},
             std::integral_constant<int, MODES>{});
    });
    constexpr int RUNALL = (RUN | (RUN << 2) | (RUN << 4) | (RUN << 6)) & ((1 << (2 * K)) - 1);
    constexpr int P0 = K % 3;  // ring phase of the first steady iteration
    for (int it = K; it < nit && !dead; it += 3) {
        iter(it, std::integral_constant<int, (P0 + 1) % 3>{}, std::integral_constant<int, P0>{},
             std::integral_constant<int, RUNALL>{});
        if (it + 1 >= nit || dead) break;
        iter(it + 1, std::integral_constant<int, (P0 + 2) % 3>{},
             std::integral_constant<int, (P0 + 1) % 3>{}, std::integral_constant<int, RUNALL>{});
        if (it + 2 >= nit || dead) break;
        iter(it + 2, std::integral_constant<int, (P0 + 3) % 3>{},
             std::integral_constant<int, (P0 + 2) % 3>{}, std::integral_constant<int, RUNALL>{});
    }
    // Row band: hand this strip's columns of the last row (n2) to the next band.
    // The table stores are plain (write-back L2), so: drain them, write the XCD's
    // L2 back (agent release), re-read the row with sc1 loads, publish
    // system-scope granules (write-through; peer HBM over xGMI when the next
    // band lives on another GPU).
    if (A.halo_out != nullptr && !dead) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const int32_t *last = A.table + A.n2 * A.pitch;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t c = c0 + 64 * k + lane;
            if (c <= A.n1) {
                const uint32_t v = (uint32_t)__hip_atomic_load(last + c, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(A.halo_out + c, ((uint64_t)A.halo_tag << 32) | v,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    if (A.trace != nullptr && lane == 0) {
        uint64_t *tr = A.trace + (int64_t)p * kTraceWords;
        tr[0] = tstart;
        tr[1] = __builtin_amdgcn_s_memrealtime();
        tr[2] = nslow;
        tr[3] = wticks;
        tr[4] = tq1;
        tr[5] = tmid;
        tr[6] = cstart;                          // shader clock (s_memtime)
        tr[7] = __builtin_amdgcn_s_memtime();
    }
}

template <int K, bool UNIT>
__global__ __launch_bounds__(64) void nw_fill_strips(FillArgs A) {
    __shared__ __attribute__((aligned(16))) int32_t lds[K * kRingWords + kRing];
    const int lane = threadIdx.x;
    for (;;) {
        uint32_t p = 0;
        if (lane == 0) p = atomicAdd(A.ctrl, 1u);
        p = __builtin_amdgcn_readfirstlane(p);
        if (p >= (uint32_t)A.nstrips) break;
        process_strip<K, UNIT>(A, lds, (int)p, lane);
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

int64_t rowpack_len(int32_t nblocks) { return kQOff + 64 * ((int64_t)nblocks + kMaxSub + 2) + 8; }

int launch_rowpack(const uint8_t *d_s2, int64_t n2, int64_t row0, uint32_t *d_q, int64_t qlen,
                   void *stream) {
    const int bs = 256;
    const int64_t nb = (qlen + bs - 1) / bs;
    hipLaunchKernelGGL(nw_rowpack, dim3((unsigned)nb), dim3(bs), 0, (hipStream_t)stream, d_s2,
                       n2, row0, d_q, qlen);
    return (int)hipGetLastError();
}

template <int K>
static void launch_k(const FillArgs &a, int grid, hipStream_t s) {
    if (a.match - a.mismatch == 1)
        hipLaunchKernelGGL((nw_fill_strips<K, true>), dim3(grid), dim3(kWave), 0, s, a);
    else
        hipLaunchKernelGGL((nw_fill_strips<K, false>), dim3(grid), dim3(kWave), 0, s, a);
}

int launch_fill(const FillArgs &a, int substrips, int grid, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (substrips) {
        case 1: launch_k<1>(a, grid, s); break;
        case 2: launch_k<2>(a, grid, s); break;
        case 4: launch_k<4>(a, grid, s); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

int lds_bytes(int substrips) { return (substrips * kRingWords + kRing) * 4; }

const char *kernel_variant() { return "superstrip-Kx64-dpp-ldsring128-gran64"; }

}  // namespace nw
