// nw_fill.hip -- gfx950 (MI355X) Needleman-Wunsch scoring-table fill.
//
// Replaces the fill loops of the reference plugins
//   src/serial/serial.cpp:21-33, src/sentinel/sentinel-mt.cpp:40-62,
//   src/idxarray/idxarray-mt.cpp:43-66
// which all compute, row-major over an int32 table of (n2+1) x (n1+1):
//   t[i][j] = max(t[i-1][j-1] + s(s1[j-1], s2[i-1]), t[i-1][j] + GAP, t[i][j-1] + GAP)
//   t[0][j] = j*GAP, t[i][0] = i*GAP                              (serial.cpp:16-17)
//
// Decomposition (DESIGN.md section 4 has the full picture):
//   * The table is cut into vertical STRIPS of 64*C columns.  Each strip is
//     swept top to bottom by one workgroup of two waves:
//       - the COMPUTE wave: lane l owns the C consecutive columns c0 + C*l + k
//         and at step s computes row i = s - l for all of them -- an
//         anti-diagonal wavefront across the lanes, a left-to-right chain of C
//         cells inside each lane.  Per cell:
//           d = diag' + s'(a, b)      v_cmp_eq_u32_sdwa (byte selects) + v_addc
//           t = max3(d, up', left')   v_max3_i32
//           u = t + GAP               v_add_u32   (u = what neighbours consume)
//         up' is the lane's own register; left'/diag' of column k > 0 are the
//         lane's own column k-1 (this step / last step).  Column 0 takes left'
//         from lane l-1's column C-1 of the previous step (DPP wave_shr:1, whose
//         "old" operand feeds lane 0 from the strip on the left) and diag' from
//         what it received the step before.  Each step's C results go to an LDS
//         ring indexed by ANTI-DIAGONAL (slot = step mod R, lane l at byte 4*C*l)
//         with one conflict-free ds_write_b(32*C).  This wave issues no table
//         stores: on gfx950 a vector store holds its wave for ~45-90 cycles.
//       - the STORE wave: row f is complete once step f + 63 is written; it
//         reads row f back from the ring (lane l: slot (f + l) mod R) and stores
//         it as ONE row-contiguous 256*C-byte segment (buffer_store_dword{,x2,x4},
//         1 KB at C = 4).  HBM sees only whole, aligned row segments.
//     The two waves are coupled by two LDS counters (steps written / rows read);
//     R = 64 + slack slots let the store wave lag by up to the slack.
//   * The strip's right column (lane 63, column C-1) is shifted into a DPP
//     wave_shl:1 register as it is computed and published per 64-row block as
//     8-byte {tag, value} granules (agent-scope atomic stores; the data is the
//     flag) for the strip to the right, which polls them -- the GPU analogue of
//     idxarray-mt's per-row progress counters (idxarray-mt.cpp:8,44,50-56).
//   * Strips are claimed from an atomic ticket in increasing order by a
//     persistent grid, so a strip's producer is always already running:
//     deadlock-free for any grid size / residency.
//   * Pure int32 VALU + LDS + HBM stores; no MFMA (there is no contraction).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "nw_internal.h"

namespace nw {

// s_memrealtime runs at 100 MHz on gfx9: 20 s watchdog for every bounded spin.
constexpr uint64_t kTimeoutTicks = 100000000ull * 20ull;
constexpr int32_t kDone = 0x7FFFFFFF;  // counter value: "no more waiting on me"

template <int C> struct Vec;
template <> struct Vec<1> { typedef int32_t T; };
template <> struct Vec<2> { typedef int32_t T __attribute__((ext_vector_type(2))); };
template <> struct Vec<4> { typedef int32_t T __attribute__((ext_vector_type(4))); };
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int C>
__device__ __forceinline__ int32_t comp(const typename Vec<C>::T &v, int k) {
    if constexpr (C == 1) {
        return v;
    } else {
        return v[k];
    }
}
template <int C>
__device__ __forceinline__ void set_comp(typename Vec<C>::T &v, int k, int32_t x) {
    if constexpr (C == 1) {
        v = x;
    } else {
        v[k] = x;
    }
}

// LDS of one workgroup: ring of R anti-diagonal slots (64*C int32 each), two
// 64-row feed buffers, the counters.
template <int C>
struct Lay {
    static constexpr int kSlot = 4 * kWave * C;       // bytes per ring slot
    // slots (64 + slack): two workgroups per CU at C = 4 and 2, four at C = 1
    static constexpr int R = C == 4 ? 76 : C == 2 ? 152 : 148;
    static constexpr int kRing = R * kSlot;          // ring bytes
    static constexpr int kFeed = kRing;              // byte offset of the feed buffers
    static constexpr int kCtl = kFeed + 2 * kWave * 4;
    static constexpr int kBytes = kCtl + 16;         // [0] steps written, [1] rows read, [2] strip
};

__device__ __forceinline__ uint64_t gran_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gran_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ctrl_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// workgroup counters in LDS (relaxed atomics: plain ds_read/ds_write that the
// compiler may neither cache nor drop)
__device__ __forceinline__ int32_t ctr_load(const int32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void ctr_store(int32_t *p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Slow path of the hand-off: re-poll until every lane's granule carries `tag`
// (s_sleep between polls).  Bounded: gives up -- raising the error word -- after
// kTimeoutTicks, or at once if another wave already raised it.  Returns the last
// value read; the caller re-checks its tag.
__device__ __noinline__ uint64_t wait_granules_slow(const uint64_t *g, uint32_t tag,
                                                    uint32_t *ctrl) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        __builtin_amdgcn_s_sleep(1);
        const uint64_t v = gran_load(g);
        if (__all((uint32_t)(v >> 32) == tag)) return v;
        if (ctrl_load(ctrl + 1) != 0u) return v;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) {
            if ((threadIdx.x & 63) == 0) atomicCAS(ctrl + 1, 0u, 1u);
            return v;
        }
    }
}

// Bounded spin until the LDS counter *p reaches `need`; returns the value seen
// (kDone once the error word is raised or the watchdog expires).
__device__ __noinline__ int32_t wait_counter(const int32_t *p, int32_t need, uint32_t *ctrl) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const int32_t v = __builtin_amdgcn_readfirstlane(ctr_load(p));
        if (v >= need) return v;
        if (ctrl_load(ctrl + 1) != 0u) return kDone;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) {
            if ((threadIdx.x & 63) == 0) atomicCAS(ctrl + 1, 0u, 3u);
            return kDone;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// Row characters of local iteration j (steps 64j .. 64j+63): lane l needs the
// bytes of rows 64j - l + u, u < 64.  rowpack16[x + kQOff] holds the 16 bytes of
// rows x .. x+15, so 4 aligned 16-byte loads cover an iteration.
__device__ __forceinline__ void load_packs(const u32x4 *__restrict__ q, int j, int lane,
                                           u32x4 (&pk)[4]) {
    const u32x4 *base = q + kQOff + (int64_t)max(j, 0) * 64 - lane;
#pragma unroll
    for (int h = 0; h < 4; ++h) pk[h] = base[16 * h];
}

// Compile-time loop: f(std::integral_constant<int, U>) for U in [B, E).
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// diag' + s'(a, b) for one cell: byte QB of the row-character word is compared
// with byte KB of the lane's packed column characters (reference match test:
// raw byte equality, serial.cpp:23-24), then
//   UNIT (match - mismatch == 1, the reference default):  d = diag' + mm' + [a == b]
//   general:                                               d = diag' + (a == b ? ms' : mm')
// (ms' / mm' have GAP pre-subtracted, because diag' = t + GAP.)  One asm
// statement per cell so hipcc keeps the compare next to its use.
template <int QB, int KB, bool UNIT>
__device__ __forceinline__ int32_t diag_plus_sub(uint32_t pk, uint32_t apk, int32_t diag,
                                                 int32_t msp, int32_t mmp) {
    int32_t d;
#ifdef NW_DBG_NOCMP
    if (true) {  // timing only: wrong scores, no VCC traffic
        d = diag + mmp + (int32_t)__builtin_amdgcn_ubfe(pk ^ apk, 8 * QB + KB, 1);
        return d;
    }
#endif
    if constexpr (UNIT) {
        asm volatile(
            "v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_%c4 src1_sel:BYTE_%c5\n\t"
            "v_addc_co_u32_e32 %0, vcc, %3, %6, vcc"
            : "=v"(d)
            : "v"(pk), "v"(apk), "v"(diag), "i"(QB), "i"(KB), "v"(mmp)
            : "vcc");
    } else {
        int32_t s;
        asm volatile(
            "v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_%c5 src1_sel:BYTE_%c6\n\t"
            "v_cndmask_b32_e32 %0, %3, %4, vcc"
            : "=v"(s)
            : "v"(pk), "v"(apk), "v"(mmp), "v"(msp), "i"(QB), "i"(KB)
            : "vcc");
        d = diag + s;
    }
    return d;
}

// Per-lane state of the compute wave on one strip.
template <int C>
struct Lanes {
    int32_t u[C];     // t + GAP of the lane's current row, column k
    int32_t dg;       // diag' of column 0 for the next step (= last step's left')
    int32_t rr;       // RAMP: row of this lane at the current step
    uint32_t apk;     // column characters of the lane, byte k = column k
    int32_t outcol;   // shift register of the strip's right column
    int32_t cb;       // last value read of the store wave's row counter
};

// 64 wavefront steps of local iteration `it` (steps s = 64*it + u, u < 64) of
// the compute wave.  Step s: compute row s - l on every lane l, write the
// results to ring slot s mod R, shift the strip's right column (lane 63's
// column C-1, row s - 63) into outcol.  After steps 4g+3 the steps-written
// counter is published; before each 4-step group the slots it overwrites are
// checked free (rows read by the store wave; the counter value was read one
// group earlier, so its LDS latency is hidden).
//   pk   : row-character words of this iteration (load_packs)
//   sb   : slot of step 64*it (= 64*it mod R)
//   gp   : where block it-1's right column goes (published after step 62, when
//          outcol holds rows 64*(it-1) .. 64*(it-1) + 63, lane l = row + l)
template <int C, bool UNIT, bool RAMP>
__device__ __forceinline__ void run_iter(char *__restrict__ lds, int it, const u32x4 (&pk)[4],
                                         int32_t msp, int32_t mmp, int32_t gap, Lanes<C> &S,
                                         int sb, uint64_t *gp, uint64_t tagw, uint32_t *ctrl,
                                         int lane) {
    typedef typename Vec<C>::T VT;
    typedef Lay<C> L;
    int32_t *ctr = (int32_t *)(lds + L::kCtl);
    const int4 *feed4 = (const int4 *)(lds + L::kFeed + ((it & 1) << 8));
    int4 fq = feed4[0];
    const int s0 = it * 64;
    static_for<0, 16>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        // ring space for steps s0+4g .. s0+4g+3: their slots held anti-diagonals
        // s - R, last needed by row s - R, so rows <= s0 + 4g + 3 - R must be read
#ifndef NW_DBG_NOFLOW
        {
            const int32_t need = s0 + 4 * g + 4 - L::R;
            if (__builtin_amdgcn_readfirstlane(S.cb) < need)
                S.cb = wait_counter(ctr + 1, need, ctrl);
            S.cb = ctr_load(ctr + 1);  // for the next group
        }
#endif
        const int4 fcur = fq;
        if constexpr (g + 1 < 16) fq = feed4[g + 1];
        const uint32_t pkw = pk[g >> 2][g & 3];
        static_for<0, 4>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            constexpr int u = 4 * g + q;
            const int32_t lf = q == 0 ? fcur.x : q == 1 ? fcur.y : q == 2 ? fcur.z : fcur.w;
            int32_t left = __builtin_amdgcn_update_dpp(lf, S.u[C - 1], 0x138 /*wave_shr:1*/,
                                                       0xF, 0xF, false);
            int32_t diag = S.dg;
            S.dg = left;
            bool act = true;
            if constexpr (RAMP) {
                S.rr += 1;
                asm volatile("" : "+v"(S.rr));  // keep the activity test in the loop
                act = S.rr >= 1;
            }
            VT tv;
            static_for<0, C>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                const int32_t d = diag_plus_sub<q, k, UNIT>(pkw, S.apk, diag, msp, mmp);
                int32_t t = max(max(d, S.u[k]), left);  // max(diag+s, up+GAP, left+GAP)
                diag = S.u[k];
                if constexpr (RAMP) {
                    // lanes still above row 1 hold row 0 (the top boundary / halo)
                    const int32_t un = act ? t + gap : S.u[k];
                    t = un - gap;
                    S.u[k] = un;
                } else {
                    S.u[k] = t + gap;
                }
                left = S.u[k];
                set_comp<C>(tv, k, t);
            });
            // ring slot (s0 + u) mod R; sb + u < R + 64 wraps at most once
            const int slot = sb + u >= L::R ? sb + u - L::R : sb + u;
            *(VT *)(lds + slot * L::kSlot + lane * (4 * C)) = tv;
            S.outcol = __builtin_amdgcn_update_dpp(comp<C>(tv, C - 1), S.outcol,
                                                   0x130 /*wave_shl:1*/, 0xF, 0xF, false);
            if constexpr (u == 62) gran_store(gp, tagw | (uint32_t)S.outcol);
#ifndef NW_DBG_NOCTRA
            if constexpr (q == 3) ctr_store(ctr, s0 + u + 1);  // steps written
#endif
        });
    });
}

// The compute wave on strip p.
template <int C, bool UNIT>
__device__ void compute_strip(const FillArgs &A, char *__restrict__ lds, int p, int lane) {
    typedef Lay<C> L;
    const int32_t gap = A.gap;
    const int32_t msp = A.match - gap, mmp = A.mismatch - gap;
    const int64_t c0 = (int64_t)p * (64 * C);
    const int64_t cl = c0 + (int64_t)C * lane;  // first column of this lane
    int32_t *ctr = (int32_t *)(lds + L::kCtl);
    bool dead = false;
    // Row 0: the boundary t[0][c] = c*GAP (serial.cpp:16), or -- for a row band
    // (mpi-horz.cpp:16-40) -- the previous band's last row, taken from its halo
    // granules once they carry this launch's tag (bounded wait).
    int32_t top[C];
#pragma unroll
    for (int k = 0; k < C; ++k) top[k] = (int32_t)((cl + k) * (int64_t)gap);
    if (A.halo_in != nullptr) {
        const uint64_t h0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            bool ok = true;
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const int64_t c = min(cl + k, A.n1);
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
    Lanes<C> S;
    S.apk = 0;
#pragma unroll
    for (int k = 0; k < C; ++k) {
        const int64_t c = cl + k;
        const uint32_t a = (c >= 1 && c <= A.n1) ? (uint32_t)A.s1[c - 1] : 0u;
        S.apk |= a << (8 * k);
        S.u[k] = top[k] + gap;  // t[0][c] + GAP
    }
    S.dg = 0;
    S.rr = -lane - 1;
    S.outcol = 0;
    S.cb = 0;

    const bool has_left = p > 0;
    const uint64_t *gin = A.gran + (int64_t)((p + A.M - 1) % A.M) * A.gstride + lane;
    uint64_t *gout = A.gran + (int64_t)(p % A.M) * A.gstride;
    const uint32_t tag_in = A.tagbase + (uint32_t)p;
    const uint64_t tagw = (uint64_t)(A.tagbase + (uint32_t)p + 1u) << 32;
    const int nblocks = A.nblocks;
    const int lastb = nblocks - 1;
    uint64_t *gscr = (uint64_t *)(A.scratch + (int64_t)blockIdx.x * kScratchWords) + lane;

    // Prefetch pipeline: the left neighbour's granules (feed) and the
    // row-character packs are loaded two iterations ahead into 3-deep register
    // rings, so no wait for a load ever falls inside the steps.  Buffer =
    // issue iteration mod 3; all loads unconditional (clamped indices).
    uint64_t gb[3];
    u32x4 pkb[3][4];
    gb[0] = gran_load(gin);                                  // block 0, for iteration 0
    gb[1] = gran_load(gin + (int64_t)min(1, lastb) * 64);    // block 1, for iteration 1
    gb[2] = 0;
    load_packs((const u32x4 *)A.rowpack, 0, lane, pkb[0]);
    load_packs((const u32x4 *)A.rowpack, 1, lane, pkb[1]);

    uint32_t nslow = 0;
    uint64_t wticks = 0;
    const uint64_t tstart = __builtin_amdgcn_s_memrealtime();
    const uint64_t cstart = __builtin_amdgcn_s_memtime();
    uint64_t tq1 = 0, tmid = 0;  // trace: times iterations nblocks/4 and nblocks/2 started

    // Iteration it: feed for block it (consumes buffer it % 3), prefetch for it+2
    // (into buffer (it+2) % 3), 64 steps, block it-1's right column published.
    // A watchdog trip marks the strip dead; it is abandoned at the boundary.
    auto iter = [&](int it, auto cons_c, auto ramp_c) {
        constexpr int CONS = decltype(cons_c)::value;  // it % 3
        constexpr int ISS = (CONS + 2) % 3;            // (it + 2) % 3
        constexpr bool RAMP = decltype(ramp_c)::value;
        if (A.trace != nullptr) {
            if (it == nblocks / 4) tq1 = __builtin_amdgcn_s_memrealtime();
            if (it == nblocks / 2) tmid = __builtin_amdgcn_s_memrealtime();
        }
        {
            int32_t fvv = kNeg;
            if (has_left && it < nblocks) {
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
            ((int32_t *)(lds + L::kFeed))[((it & 1) << 6) + lane] = fvv;
        }
        gb[ISS] = gran_load(gin + (int64_t)min(it + 2, lastb) * 64);
        load_packs((const u32x4 *)A.rowpack, it + 2, lane, pkb[ISS]);
        const int b = it - 1;  // block whose right column this iteration publishes
        uint64_t *gp = (b >= 0 && b < nblocks) ? gout + (int64_t)b * 64 + lane : gscr;
        const int sb = __builtin_amdgcn_readfirstlane((int)(((uint32_t)it * 64u) % (uint32_t)L::R));
        run_iter<C, UNIT, RAMP>(lds, it, pkb[CONS], msp, mmp, gap, S, sb, gp, tagw, A.ctrl, lane);
    };
    // iteration 0 ramps the wavefront in (lanes above row 1 hold row 0); row
    // 64*nblocks - 1 completes (lane 63) at step 64*nblocks + 62, iteration nblocks
    const int nit = nblocks + 1;
    iter(0, std::integral_constant<int, 0>{}, std::true_type{});
    for (int it = 1; it < nit && !dead; it += 3) {
        iter(it, std::integral_constant<int, 1>{}, std::false_type{});
        if (it + 1 >= nit || dead) break;
        iter(it + 1, std::integral_constant<int, 2>{}, std::false_type{});
        if (it + 2 >= nit || dead) break;
        iter(it + 2, std::integral_constant<int, 0>{}, std::false_type{});
    }
    // every row is in the ring (or the strip is abandoned): release the store wave
    ctr_store(ctr, kDone);
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

// The store wave on strip p: rows 0 .. n2 leave the ring as whole row segments.
// One 16-byte-per-lane store covers NR = 4/C rows (1 KB: a row of a C = 4 strip,
// two rows of a C = 2 strip): B-lane l takes row f + l / (16C), columns
// 4 * (l % (16C)) .. +3, i.e. the pieces of the NR compute lanes
// a = NR * (l % (16C)) + m that wrote them, each in slot (row + a) mod R.
// Rows go in batches of BATCH: wait until the compute wave has written them,
// read the whole batch from the ring, store it, then release its slots.
template <int C>
__device__ void store_strip(const FillArgs &A, char *__restrict__ lds, int p, int lane) {
    typedef typename Vec<C>::T VT;
    typedef Lay<C> L;
    constexpr int NR = 4 / C;                  // rows per store instruction
    constexpr int Q = 16 * C;                  // lanes per row
    constexpr int BATCH = C == 4 ? 4 : 16;     // rows per batch (ring slack: R - 64)
    constexpr int NG = BATCH / NR;             // stores per batch
    constexpr uint32_t kRingB = (uint32_t)L::kRing;
    int32_t *ctr = (int32_t *)(lds + L::kCtl);
    const int64_t c0 = (int64_t)p * (64 * C);
    const int32_t nrows = (int32_t)(A.n2 + 1);
    const bool timing = (A.flags & 1) != 0;
    const int ro = lane / Q, cq = lane % Q;
    const bool col_ok = c0 + 4 * cq < A.pitch;  // the last strip may overhang the pitch
    const int64_t rowb = timing ? 0 : A.pitch * 4;
    char *scr = (char *)(A.scratch + (int64_t)blockIdx.x * kScratchWords);
    char *rowp = timing ? scr : (char *)(A.table + c0);
    const uint32_t voff = (uint32_t)(ro * rowb) + (uint32_t)cq * 16u;
    uint32_t pa[NR];  // ring byte address of piece m of this lane's row
#pragma unroll
    for (int m = 0; m < NR; ++m) {
        const int a = NR * cq + m;
        pa[m] = (uint32_t)((ro + a) % L::R) * L::kSlot + (uint32_t)a * (4u * C);
    }
    auto adv = [&](uint32_t x) {  // NR rows further down the ring
        x += NR * L::kSlot;
        return x >= kRingB ? x - kRingB : x;
    };
    int32_t avail = 0;  // rows complete in the ring (steps written - 63)
#ifdef NW_DBG_BFREE
    ctr_store(ctr + 1, kDone);
    return;
#endif
    for (int32_t f = 0; f < nrows; f += BATCH) {
        const int32_t want = min(f + BATCH, nrows);
        if (avail < want) {
            int32_t sa = __builtin_amdgcn_readfirstlane(ctr_load(ctr));
            if (sa != kDone && sa - 63 < want) sa = wait_counter(ctr, want + 63, A.ctrl);
            avail = sa == kDone ? nrows : min(sa - 63, nrows);
        }
        u32x4 v[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
#pragma unroll
            for (int m = 0; m < NR; ++m) {
                const VT x = *(const VT *)(lds + pa[m]);
                pa[m] = adv(pa[m]);
#pragma unroll
                for (int k = 0; k < C; ++k) v[g][m * C + k] = (uint32_t)comp<C>(x, k);
            }
        }
#ifdef NW_DBG_BNOSTORE
        if (v[0][0] == 0x12345678u && v[NG - 1][3] == 0x9abcdefu) *(u32x4 *)scr = v[0];
#else
        if (want - f == BATCH) {
#pragma unroll
            for (int g = 0; g < NG; ++g)
                if (col_ok) *(u32x4 *)(rowp + (int64_t)g * NR * rowb + voff) = v[g];
        } else {
#pragma unroll
            for (int g = 0; g < NG; ++g)
                if (col_ok && f + g * NR + ro < nrows)
                    *(u32x4 *)(rowp + (int64_t)g * NR * rowb + voff) = v[g];
        }
#endif
        rowp += BATCH * rowb;
        ctr_store(ctr + 1, want);  // rows read: their slots may be overwritten
    }
    ctr_store(ctr + 1, kDone);
    // Row band: hand this strip's columns of the last row (n2) to the next band.
    // The table stores are plain (write-back L2), so: drain them, write the XCD's
    // L2 back (agent release), re-read the row with sc1 loads, publish
    // system-scope granules (write-through; peer HBM over xGMI when the next
    // band lives on another GPU).
    if (A.halo_out != nullptr && ctrl_load(A.ctrl + 1) == 0u) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const int32_t *last = A.table + A.n2 * A.pitch;
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const int64_t c = c0 + (int64_t)C * lane + k;
            if (c <= A.n1) {
                const uint32_t x = (uint32_t)__hip_atomic_load(last + c, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(A.halo_out + c, ((uint64_t)A.halo_tag << 32) | x,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// Persistent grid of two-wave workgroups: wave 0 computes, wave 1 stores.
template <int C, bool UNIT>
__global__ __launch_bounds__(128) void nw_fill_strips(FillArgs A) {
    typedef Lay<C> L;
    __shared__ __attribute__((aligned(16))) char lds[L::kBytes];
    int32_t *ctr = (int32_t *)(lds + L::kCtl);
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    for (;;) {
        if (threadIdx.x == 0) {
            ctr[0] = 0;
            ctr[1] = 0;
            ctr[2] = (int32_t)atomicAdd(A.ctrl, 1u);
        }
        __syncthreads();
        const int p = __builtin_amdgcn_readfirstlane(ctr[2]);
        if (p >= A.nstrips) break;
        if (wave == 0)
            compute_strip<C, UNIT>(A, lds, p, lane);
        else
            store_strip<C>(A, lds, p, lane);
        __syncthreads();  // the ring and counters are reused by the next strip
    }
}

// rowpack16[idx] = B[x .. x+15] (16 bytes), x = idx - kQOff, B[y] = s2[row0 + y - 1]
// for 1 <= y <= n2 (local rows of this launch), else 0.
__global__ void nw_rowpack(const uint8_t *__restrict__ s2, int64_t n2, int64_t row0,
                           u32x4 *__restrict__ q, int64_t qlen) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= qlen) return;
    const int64_t x = idx - kQOff;
    u32x4 v = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int64_t y = x + k;
        const uint32_t b = (y >= 1 && y <= n2) ? (uint32_t)s2[row0 + y - 1] : 0u;
        v[k >> 2] |= b << (8 * (k & 3));
    }
    q[idx] = v;
}

// entries of 16 bytes: iteration j <= nblocks + 2 (prefetch of the last one)
// reads up to index kQOff + 64 * (nblocks + 2) + 48
int64_t rowpack_len(int32_t nblocks) { return kQOff + 64 * ((int64_t)nblocks + 3) + 16; }

int launch_rowpack(const uint8_t *d_s2, int64_t n2, int64_t row0, void *d_q, int64_t qlen,
                   void *stream) {
    const int bs = 256;
    const int64_t nb = (qlen + bs - 1) / bs;
    hipLaunchKernelGGL(nw_rowpack, dim3((unsigned)nb), dim3(bs), 0, (hipStream_t)stream, d_s2,
                       n2, row0, (u32x4 *)d_q, qlen);
    return (int)hipGetLastError();
}

template <int C>
static void launch_c(const FillArgs &a, int grid, hipStream_t s) {
    if (a.match - a.mismatch == 1)
        hipLaunchKernelGGL((nw_fill_strips<C, true>), dim3(grid), dim3(2 * kWave), 0, s, a);
    else
        hipLaunchKernelGGL((nw_fill_strips<C, false>), dim3(grid), dim3(2 * kWave), 0, s, a);
}

int launch_fill(const FillArgs &a, int substrips, int grid, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (substrips) {
        case 1: launch_c<1>(a, grid, s); break;
        case 2: launch_c<2>(a, grid, s); break;
        case 4: launch_c<4>(a, grid, s); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

int lds_bytes(int substrips) {
    switch (substrips) {
        case 1: return Lay<1>::kBytes;
        case 2: return Lay<2>::kBytes;
        default: return Lay<4>::kBytes;
    }
}

const char *kernel_variant() { return "strip-64xC-computewave+storewave-diagring-rowflush-gran64"; }

}  // namespace nw
