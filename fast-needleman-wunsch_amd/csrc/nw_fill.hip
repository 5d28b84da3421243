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
constexpr int kStoreWaves = 2;         // store waves per strip workgroup
#ifndef NW_BCAP
#define NW_BCAP 0  // max older stores a store wave keeps in flight (0: no cap)
#endif

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
    // counters: [0] steps written, [1 + b] rows read by store wave b, [3] strip
    static constexpr int kBytes = kCtl + 16;
    // compute wave: check ring space every kChk steps, publish progress every
    // kPub steps (coarse only where the slack R - 64 allows it)
    static constexpr int kChk = R - 64 >= 48 ? 16 : 4;
    static constexpr int kPub = R - 64 >= 48 ? 8 : 4;
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

// Slow path of the hand-off: re-poll the granules of one 64-row block until
// those of chunk c (lanes 16c .. 16c+15) carry `tag` (s_sleep between polls).
// Bounded: gives up -- raising the error word -- after kTimeoutTicks, or at once
// if another wave already raised it.  Returns the last value read; the caller
// re-checks its tag.
__device__ __noinline__ uint64_t wait_chunk(const uint64_t *g, uint32_t tag, int c,
                                            uint32_t *ctrl) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x & 63;
    const bool in_chunk = (lane >> 4) == c;
    for (;;) {
        __builtin_amdgcn_s_sleep(1);
        const uint64_t v = gran_load(g);
        if (__all(!in_chunk || (uint32_t)(v >> 32) == tag)) return v;
        if (ctrl_load(ctrl + 1) != 0u) return v;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) {
            if (lane == 0) atomicCAS(ctrl + 1, 0u, 1u);
            return v;
        }
    }
}

// Leading 16-row chunks of a block whose granules all carry `tag` (0 .. 4).
__device__ __forceinline__ int chunks_ready(uint64_t v, uint32_t tag) {
    const uint64_t ok = __ballot((uint32_t)(v >> 32) == tag);
    int n = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c)
        if (n == c && ((ok >> (16 * c)) & 0xFFFFull) == 0xFFFFull) n = c + 1;
    return n;
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

// Rows every store wave has read out of the ring (each publishes the start of
// its next batch; all rows below the smallest are out).
__device__ __forceinline__ int32_t rows_read(const int32_t *ctr) {
    int32_t v = ctr_load(ctr + 1);
#pragma unroll
    for (int b = 1; b < kStoreWaves; ++b) v = min(v, ctr_load(ctr + 1 + b));
    return v;
}
__device__ __forceinline__ void wait_rows_read(const int32_t *ctr, int32_t need, uint32_t *ctrl) {
#pragma unroll
    for (int b = 0; b < kStoreWaves; ++b) (void)wait_counter(ctr + 1 + b, need, ctrl);
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

// How a cell's substitution score is formed.
//   SUB_PROF : query profile -- the row word holds s(a_k, b) - GAP per row as
//              int8 (one profile per distinct column character, nw_profile);
//              d = diag' + sext(byte):  ONE v_add_u32_sdwa, no compare
//   SUB_UNIT : match - mismatch == 1: d = diag' + mm' + [a == b]
//              (v_cmp_eq_u32_sdwa -> vcc -> v_addc)
//   SUB_GEN  : d = diag' + (a == b ? ms' : mm')  (v_cmp -> vcc -> v_cndmask, add)
// The compare forms test raw byte equality, the reference's match test
// (serial.cpp:23-24); ms' / mm' / the profile bytes have GAP pre-subtracted
// because diag' = t + GAP.  On a lone gfx950 wave the vcc round trip costs
// ~15 cycles per cell, which is why the profile form exists.
enum Sub { SUB_PROF = 0, SUB_UNIT = 1, SUB_GEN = 2 };

template <int QB, int KB, int MODE>
__device__ __forceinline__ int32_t diag_plus_sub(uint32_t pk, uint32_t apk, int32_t diag,
                                                 int32_t msp, int32_t mmp) {
    int32_t d;
    if constexpr (MODE == SUB_PROF) {
        asm("v_add_u32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD "
            "src0_sel:DWORD src1_sel:BYTE_%c3"
            : "=v"(d)
            : "v"(diag), "v"(pk), "i"(QB));
    } else if constexpr (MODE == SUB_UNIT) {
        asm volatile(
            "v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_%c4 src1_sel:BYTE_%c5\n\t"
            "v_addc_co_u32_e32 %0, vcc, %3, %6, vcc"
            : "=v"(d)
            : "v"(pk), "v"(apk), "v"(diag), "i"(QB), "i"(KB), "v"(mmp)
            : "vcc");
    } else {
        int32_t sc;
        asm volatile(
            "v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_%c5 src1_sel:BYTE_%c6\n\t"
            "v_cndmask_b32_e32 %0, %3, %4, vcc"
            : "=v"(sc)
            : "v"(pk), "v"(apk), "v"(mmp), "v"(msp), "i"(QB), "i"(KB)
            : "vcc");
        d = diag + sc;
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

// The feed of one iteration: the left neighbour's right column for rows
// 64*it .. 64*it+63, published there in 16-row chunks.  `ready` leading chunks
// were found published when the iteration started; before the group that
// first reads chunk c >= ready, run_iter waits for it (wait_chunk) and writes
// its 16 feed values.
struct Feed {
    const uint64_t *g;  // this lane's granule of the block (left neighbour's slot)
    uint32_t tag;
    int ready;
    int32_t gap;
    uint32_t nslow;
    uint64_t wticks;
    bool dead;
    bool trace_pub;     // debug trace: stamp the publish of chunk 0 in this iteration
    uint64_t tpub;
};

// Row words per lane and iteration: one per column of the lane in the profile
// form (each column has its own character's profile), one in the compare forms.
template <int C, int MODE>
constexpr int npk() { return MODE == SUB_PROF ? C : 1; }

// 64 wavefront steps of local iteration `it` (steps s = 64*it + u, u < 64) of
// the compute wave.  Step s: compute row s - l on every lane l, write the
// results to ring slot s mod R, shift the strip's right column (lane 63's
// column C-1, row s - 63) into outcol.  Every kPub steps the steps-written
// counter is published; every kChk steps the slots the next kChk overwrite are
// checked free (rows read by the store wave; the counter value was read kChk
// steps earlier, so its LDS latency is hidden).
//   pk   : row words of this iteration (load_packs), [npk][4] x 16 rows each
//   sb   : slot of step 64*it (= 64*it mod R)
//   gp   : this lane's granule of block it-1 (the right column is published in
//          16-row chunks, after steps 14, 30, 46, 62)
//   F    : the feed of this iteration (chunks not yet published are waited for)
template <int C, int MODE, bool RAMP>
__device__ __forceinline__ void run_iter(char *__restrict__ lds, int it,
                                         const u32x4 (&pk)[npk<C, MODE>()][4], int32_t msp,
                                         int32_t mmp, int32_t gap, Lanes<C> &S, int sb,
                                         uint64_t *gp, uint64_t tagw, uint32_t *ctrl, Feed &F,
                                         int lane) {
    typedef typename Vec<C>::T VT;
    typedef Lay<C> L;
    int32_t *ctr = (int32_t *)(lds + L::kCtl);
    const int4 *feed4 = (const int4 *)(lds + L::kFeed + ((it & 1) << 8));
    int4 fq = feed4[0];
    const int s0 = it * 64;
    static_for<0, 16>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        // ring space for steps s0+4g .. s0+4g+kChk-1: their slots held
        // anti-diagonals s - R, last needed by row s - R, so rows
        // <= s0 + 4g + kChk - 1 - R must have been read
        if constexpr ((4 * g) % L::kChk == 0) {
            const int32_t need = s0 + 4 * g + L::kChk - L::R;
            if (__builtin_amdgcn_readfirstlane(S.cb) < need) wait_rows_read(ctr, need, ctrl);
            S.cb = rows_read(ctr);  // for the next check (kChk steps on)
        }
        // chunk (g+1)/4 is read by the feed load below: wait for it if it was
        // not yet published when the iteration started
        if constexpr ((g & 3) == 3 && g + 1 < 16) {
            constexpr int c = (g + 1) >> 2;
            if (F.ready <= c) {
                const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
                const uint64_t v = wait_chunk(F.g, F.tag, c, ctrl);
                F.dead |= !__all((lane >> 4) != c || (uint32_t)(v >> 32) == F.tag);
                F.nslow += 1;
                F.wticks += __builtin_amdgcn_s_memrealtime() - w0;
                if ((lane >> 4) == c)
                    ((int32_t *)(lds + L::kFeed))[((it & 1) << 6) + lane] =
                        (int32_t)(uint32_t)v + F.gap;
                F.ready = c + 1;
            }
        }
        const int4 fcur = fq;
        if constexpr (g + 1 < 16) fq = feed4[g + 1];
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
                const uint32_t pkw = pk[MODE == SUB_PROF ? k : 0][g >> 2][g & 3];
                const int32_t d = diag_plus_sub<q, k, MODE>(pkw, S.apk, diag, msp, mmp);
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
            // after step 14 + 16c outcol's lanes 48..63 hold rows 64(it-1) + 16c + 0..15
            // of the right column: publish that chunk (lane l -> row 64(it-1) + l - 48 + 16c)
            if constexpr ((u & 15) == 14) {
                if (lane >= 48) gran_store(gp + (16 * (u >> 4) - 48), tagw | (uint32_t)S.outcol);
                if constexpr (u == 14) {
                    if (F.trace_pub) F.tpub = __builtin_amdgcn_s_memrealtime();
                }
            }
            if constexpr ((u + 1) % L::kPub == 0) ctr_store(ctr, s0 + u + 1);  // steps written
        });
    });
}

// The compute wave on strip p.
template <int C, int MODE>
__device__ void compute_strip(const FillArgs &A, char *__restrict__ lds, int p, int lane) {
    typedef Lay<C> L;
    constexpr int NPK = npk<C, MODE>();
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

    // Row words: the raw s2 bytes (compare forms), or per column k the profile
    // of the lane's character a_k (profile form; nw_profile).
    const u32x4 *pkp[NPK];
    if constexpr (MODE == SUB_PROF) {
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const uint32_t m = min((uint32_t)A.charmap[(S.apk >> (8 * k)) & 255u], kMaxProf - 1u);
            pkp[k] = (const u32x4 *)A.prof + (int64_t)m * A.prof_stride;
        }
    } else {
        pkp[0] = (const u32x4 *)A.rowpack;
    }
    // Prefetch pipeline: the left neighbour's granules (feed) and the row words
    // are loaded PD iterations ahead into (PD+1)-deep register rings, so no wait
    // for a load falls inside the steps (PD = 2; 1 when four profile words per
    // iteration would not fit in registers).  Buffer = iteration mod NB; all
    // loads unconditional (clamped indices).
    constexpr int NB = NPK >= 4 ? 2 : 3, PD = NB - 1;
    uint64_t gb[NB];
    u32x4 pkb[NB][NPK][4];
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        gb[i] = gran_load(gin + (int64_t)min(i, lastb) * 64);  // block i, for iteration i
#pragma unroll
        for (int k = 0; k < NPK; ++k) load_packs(pkp[k], i, lane, pkb[i][k]);
    }

    Feed F;
    F.tag = tag_in;
    F.gap = gap;
    F.nslow = 0;
    F.wticks = 0;
    F.dead = dead;  // (a halo wait may already have given up)
    const uint64_t tstart = __builtin_amdgcn_s_memrealtime();
    const uint64_t cstart = __builtin_amdgcn_s_memtime();
    uint64_t tq1 = 0, tmid = 0;  // trace: times iterations nblocks/4 and nblocks/2 started
    uint64_t tpub = 0, tsee = 0, twait = 0;  // trace: publish / see / wait start, block nblocks/2 chunk 0
    F.trace_pub = false;
    F.tpub = 0;

    // Iteration it: feed for block it (consumes buffer it % 3), prefetch for it+2
    // (into buffer (it+2) % 3), 64 steps, block it-1's right column published.
    // A watchdog trip marks the strip dead; it is abandoned at the boundary.
    auto iter = [&](int it, auto cons_c, auto ramp_c) {
        constexpr int CONS = decltype(cons_c)::value;  // it % NB
        constexpr int ISS = (CONS + PD) % NB;          // (it + PD) % NB
        constexpr bool RAMP = decltype(ramp_c)::value;
        if (A.trace != nullptr) {
            if (it == nblocks / 4) tq1 = __builtin_amdgcn_s_memrealtime();
            if (it == nblocks / 2) tmid = __builtin_amdgcn_s_memrealtime();
            F.trace_pub = it == nblocks / 2 + 1;
        }
        {
            int32_t fvv = kNeg;
            F.ready = 4;
            if (has_left && it < nblocks) {
                uint64_t gv = gb[CONS];  // block it, loaded PD iterations ago
                F.g = gin + (int64_t)it * 64;
                F.ready = chunks_ready(gv, tag_in);
                if (F.ready == 0) {  // chunk 0 is needed right away
                    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
                    if (A.trace != nullptr && it == nblocks / 2) twait = w0;
                    gv = wait_chunk(F.g, tag_in, 0, A.ctrl);
                    F.dead |= !__all((lane >> 4) != 0 || (uint32_t)(gv >> 32) == tag_in);
                    F.nslow += 1;
                    F.wticks += __builtin_amdgcn_s_memrealtime() - w0;
                    F.ready = max(1, chunks_ready(gv, tag_in));
                }
                fvv = (int32_t)(uint32_t)gv + gap;
                if (A.trace != nullptr && it == nblocks / 2) tsee = __builtin_amdgcn_s_memrealtime();
            }
            ((int32_t *)(lds + L::kFeed))[((it & 1) << 6) + lane] = fvv;
        }
        gb[ISS] = gran_load(gin + (int64_t)min(it + PD, lastb) * 64);
#pragma unroll
        for (int k = 0; k < NPK; ++k) load_packs(pkp[k], it + PD, lane, pkb[ISS][k]);
        const int b = it - 1;  // block whose right column this iteration publishes
        uint64_t *gp = (b >= 0 && b < nblocks) ? gout + (int64_t)b * 64 + lane : gscr;
        const int sb = __builtin_amdgcn_readfirstlane((int)(((uint32_t)it * 64u) % (uint32_t)L::R));
        run_iter<C, MODE, RAMP>(lds, it, pkb[CONS], msp, mmp, gap, S, sb, gp, tagw, A.ctrl, F,
                                lane);
        dead = F.dead;
    };
    // iteration 0 ramps the wavefront in (lanes above row 1 hold row 0); row
    // 64*nblocks - 1 completes (lane 63) at step 64*nblocks + 62, iteration nblocks
    const int nit = nblocks + 1;
    iter(0, std::integral_constant<int, 0>{}, std::true_type{});
    for (int it = 1; it < nit && !dead; it += NB) {
        iter(it, std::integral_constant<int, 1 % NB>{}, std::false_type{});
        if (it + 1 >= nit || dead) break;
        iter(it + 1, std::integral_constant<int, 2 % NB>{}, std::false_type{});
        if constexpr (NB == 3) {
            if (it + 2 >= nit || dead) break;
            iter(it + 2, std::integral_constant<int, 0>{}, std::false_type{});
        }
    }
    // every row is in the ring (or the strip is abandoned): release the store wave
    ctr_store(ctr, kDone);
    if (A.trace != nullptr && lane == 0) {
        uint64_t *tr = A.trace + (int64_t)p * kTraceWords;
        tr[0] = tstart;
        tr[1] = __builtin_amdgcn_s_memrealtime();
        tr[2] = F.nslow;
        tr[3] = F.wticks;
        tr[4] = tq1;
        tr[5] = tmid;
        tr[6] = cstart;                          // shader clock (s_memtime)
        tr[7] = __builtin_amdgcn_s_memtime();
        tr[8] = F.tpub;
        tr[9] = tsee;
        tr[10] = twait;
    }
}

// The store wave on strip p: rows 0 .. n2 leave the ring as whole row segments.
// One 16-byte-per-lane store covers NR = 4/C rows (1 KB: a row of a C = 4 strip,
// two rows of a C = 2 strip): B-lane l takes row f + l / (16C), columns
// 4 * (l % (16C)) .. +3, i.e. the pieces of the NR compute lanes
// a = NR * (l % (16C)) + m that wrote them, each in slot (row + a) mod R.
// Rows go in batches of BATCH, dealt round robin to the kStoreWaves store waves
// (b = this wave): wait until the compute wave has written the batch, read it
// from the ring, store it, then release its slots.  Under full HBM load one
// store instruction holds its wave for ~190 cycles, which is why one compute
// wave has several store waves.
template <int C>
__device__ void store_strip(const FillArgs &A, char *__restrict__ lds, int p, int lane, int b) {
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
    const int32_t f0 = b * BATCH;
    char *rowp = timing ? scr : (char *)(A.table + c0) + (int64_t)f0 * rowb;
    const uint32_t voff = (uint32_t)(ro * rowb) + (uint32_t)cq * 16u;
    uint32_t pa[NR];  // ring byte address of piece m of this lane's row
#pragma unroll
    for (int m = 0; m < NR; ++m) {
        const int a = NR * cq + m;
        pa[m] = (uint32_t)((f0 + ro + a) % L::R) * L::kSlot + (uint32_t)a * (4u * C);
    }
    auto adv = [&](uint32_t x, uint32_t rows) {  // `rows` (< R) rows further down the ring
        x += rows * L::kSlot;
        return x >= kRingB ? x - kRingB : x;
    };
    int32_t *mine = ctr + 1 + b;
    int32_t avail = 0;  // rows complete in the ring (steps written - 63)
    for (int32_t f = f0; f < nrows; f += kStoreWaves * BATCH) {
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
                pa[m] = adv(pa[m], NR);
#pragma unroll
                for (int k = 0; k < C; ++k) v[g][m * C + k] = (uint32_t)comp<C>(x, k);
            }
        }
#pragma unroll
        for (int m = 0; m < NR; ++m) pa[m] = adv(pa[m], (kStoreWaves - 1) * BATCH);  // skip the others'
#if NW_BCAP > 0
        // keep this CU's store queue short: the compute wave's hand-off polls
        // wait behind it (vmcnt: vmcnt[3:0] | vmcnt[5:4] << 14, others maxed)
        __builtin_amdgcn_s_waitcnt((NW_BCAP & 15) | (7 << 4) | (15 << 8) | ((NW_BCAP >> 4) << 14));
#endif
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
        rowp += kStoreWaves * BATCH * rowb;
        ctr_store(mine, f + kStoreWaves * BATCH);  // my rows below are out of the ring
    }
    ctr_store(mine, kDone);
    // Row band: hand this strip's columns of the last row (n2) to the next band.
    // The table stores are plain (write-back L2), so: drain them, write the XCD's
    // L2 back (agent release), re-read the row with sc1 loads, publish
    // system-scope granules (write-through; peer HBM over xGMI when the next
    // band lives on another GPU).
    // (the store wave that stored row n2 does it)
    if (A.halo_out != nullptr && ((nrows - 1) / BATCH) % kStoreWaves == b &&
        ctrl_load(A.ctrl + 1) == 0u) {
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

// Persistent grid of workgroups of 1 + kStoreWaves waves: wave 0 computes,
// the others store.
template <int C, bool UNIT>
__global__ __launch_bounds__(64 * (1 + kStoreWaves)) void nw_fill_strips(FillArgs A) {
    typedef Lay<C> L;
    __shared__ __attribute__((aligned(16))) char lds[L::kBytes];
    int32_t *ctr = (int32_t *)(lds + L::kCtl);
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    for (;;) {
        if (threadIdx.x == 0) {
            for (int b = 0; b < 1 + kStoreWaves; ++b) ctr[b] = 0;
            ctr[3] = (int32_t)atomicAdd(A.ctrl, 1u);
        }
        __syncthreads();
        const int p = __builtin_amdgcn_readfirstlane(ctr[3]);
        if (p >= A.nstrips) break;
        if (wave == 0) {
            // profile form when the launch's profiles exist (nprof of them, built
            // by nw_profile from the column characters), else the compares
            const uint32_t np = __builtin_amdgcn_readfirstlane(ctrl_load(A.nprof));
            if (A.prof != nullptr && np >= 1u && np <= kMaxProf)
                compute_strip<C, SUB_PROF>(A, lds, p, lane);
            else if (UNIT)
                compute_strip<C, SUB_UNIT>(A, lds, p, lane);
            else
                compute_strip<C, SUB_GEN>(A, lds, p, lane);
        } else
            store_strip<C>(A, lds, p, lane, wave - 1);
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

// Column-character map of a launch (one workgroup): which byte values occur in
// s1, in increasing order -> charmap[c] = profile index (0xFF: absent),
// chars[m] = the character of profile m (m < kMaxProf), *nprof = how many
// distinct characters s1 holds.
__global__ __launch_bounds__(1024) void nw_charmap(const uint8_t *__restrict__ s1, int64_t n1,
                                                   uint8_t *__restrict__ charmap,
                                                   uint8_t *__restrict__ chars,
                                                   uint32_t *__restrict__ nprof) {
    __shared__ uint32_t present[8];
    __shared__ uint32_t before[8];
    if (threadIdx.x < 8) present[threadIdx.x] = 0;
    __syncthreads();
    uint32_t mine[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t i = threadIdx.x; i < n1; i += blockDim.x) {
        const uint32_t c = s1[i];
        mine[c >> 5] |= 1u << (c & 31);
    }
#pragma unroll
    for (int w = 0; w < 8; ++w)
        if (mine[w]) atomicOr(&present[w], mine[w]);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int w = 0; w < 8; ++w) {
            before[w] = acc;
            acc += (uint32_t)__builtin_popcount(present[w]);
        }
        *nprof = acc;
    }
    __syncthreads();
    if (threadIdx.x < 256) {
        const uint32_t c = threadIdx.x, w = c >> 5, bit = 1u << (c & 31);
        const uint32_t idx = before[w] + (uint32_t)__builtin_popcount(present[w] & (bit - 1u));
        const bool here = (present[w] & bit) != 0u;
        charmap[c] = here ? (uint8_t)min(idx, 255u) : (uint8_t)0xFF;
        if (here && idx < kMaxProf) chars[idx] = (uint8_t)c;
    }
}

// Query profiles (SUB_PROF): prof[m * qlen + idx] = 16 int8 of
// s(chars[m], B[x + k]) - GAP, k < 16, x = idx - kQOff, B[y] = s2[row0 + y - 1]
// for 1 <= y <= n2 (else 0) -- the rowpack16 layout with the substitution score
// of column character chars[m] against every row already applied.
__global__ void nw_profile(const uint8_t *__restrict__ s2, int64_t n2, int64_t row0,
                           const uint8_t *__restrict__ chars, const uint32_t *__restrict__ nprof,
                           int32_t match, int32_t mismatch, int32_t gap, u32x4 *__restrict__ prof,
                           int64_t qlen) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t m = blockIdx.y;
    if (idx >= qlen || m >= *nprof) return;
    const uint32_t a = chars[m];
    const int64_t x = idx - kQOff;
    u32x4 v = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int64_t y = x + k;
        const uint32_t b = (y >= 1 && y <= n2) ? (uint32_t)s2[row0 + y - 1] : 0u;
        const uint32_t sc = (uint32_t)((a == b ? match : mismatch) - gap) & 255u;
        v[k >> 2] |= sc << (8 * (k & 3));
    }
    prof[(int64_t)m * qlen + idx] = v;
}

int launch_profiles(const uint8_t *d_s1, int64_t n1, const uint8_t *d_s2, int64_t n2,
                    int64_t row0, int32_t match, int32_t mismatch, int32_t gap, uint8_t *meta,
                    void *d_prof, int64_t qlen, void *stream) {
    uint8_t *charmap = meta, *chars = meta + 256;
    uint32_t *nprof = (uint32_t *)(meta + 256 + kMaxProf);
    hipLaunchKernelGGL(nw_charmap, dim3(1), dim3(1024), 0, (hipStream_t)stream, d_s1, n1, charmap,
                       chars, nprof);
    const int bs = 256;
    const int64_t nb = (qlen + bs - 1) / bs;
    hipLaunchKernelGGL(nw_profile, dim3((unsigned)nb, kMaxProf), dim3(bs), 0, (hipStream_t)stream,
                       d_s2, n2, row0, chars, nprof, match, mismatch, gap, (u32x4 *)d_prof, qlen);
    return (int)hipGetLastError();
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
        hipLaunchKernelGGL((nw_fill_strips<C, true>), dim3(grid), dim3((1 + kStoreWaves) * kWave), 0, s, a);
    else
        hipLaunchKernelGGL((nw_fill_strips<C, false>), dim3(grid), dim3((1 + kStoreWaves) * kWave), 0, s, a);
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
