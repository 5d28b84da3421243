// nw_rows.hip -- gfx950 (MI355X) row-scan PANEL fill: the second kernel family
// behind the same launch (nw_params.kernel = NW_KERNEL_ROWS).
//
// Same table as the strip kernel (nw_fill.hip) and the reference fills
//   src/serial/serial.cpp:21-33, src/sentinel/sentinel-mt.cpp:40-62,
//   src/idxarray/idxarray-mt.cpp:43-66
//   t[i][j] = max(t[i-1][j-1] + s(s1[j-1], s2[i-1]), t[i-1][j] + GAP, t[i][j-1] + GAP)
// but a wave holds a ROW, not an anti-diagonal.  With x = t - GAP*(i+j) (the w
// form, in which both gap terms vanish)
//   x[i][j] = max(x[i-1][j-1] + s - 2 GAP, x[i-1][j], x[i][j-1]),
// so once b_j = max(x[i-1][j-1] + s', x[i-1][j]) is known for the whole row
// (it only reads row i-1), the row itself is a PREFIX MAXIMUM of b along j,
// seeded with the left neighbour's value:
//   * lane l of a compute wave owns C consecutive columns: local prefix (C-1
//     v_max3 on the chain), then
//   * an inclusive max-scan of the lane totals over the 64 lanes: six
//     v_max_i32_dpp (row_shr:1,2,4,8, row_bcast:15, row_bcast:31), then
//   * the exclusive carry (one DPP wave_shr:1 whose "old" operand is the left
//     neighbour's value) folded into the lane's other columns.
// A row of 64*C cells is therefore complete -- and leaves as ONE row-contiguous
// 256*C-byte segment -- right after it is computed: there is no anti-diagonal
// skew, so the LDS ring between the compute wave and its store wave holds
// kR = 32 rows (vs 128 anti-diagonal slots), and a workgroup can run several
// wide compute waves (4 x 256 columns) where the strip kernel fits one.  The
// left neighbour's value of row i is needed only at the carry step, so a
// panel trails its left neighbour by a few rows instead of 64 per wave.
//
// Smith-Waterman (config 5) in the same shape: with u = t - GAP*j the 0 floor
// becomes z_j = -GAP*j, increasing along the row, so
//   u[i][j] = max(u[i-1][j-1] + s - GAP, u[i-1][j] + GAP, z_j, u[i][j-1])
// is again a prefix maximum (z_j dominates every earlier z).
//
// Decomposition:
//   * PANELS of P = NW*64*C columns, claimed in order from an atomic ticket
//     by a persistent grid (one workgroup per CU): a panel's producer is
//     always already running (deadlock-free for any grid / residency), the GPU
//     analogue of idxarray-mt's progress counters (idxarray-mt.cpp:8,44,50-56).
//   * A workgroup = NW compute waves (wave w: columns w*64C .. +64C-1 of the
//     panel), kSPW store waves per compute wave (batches of its ring dealt
//     round robin), a feeder-in and a feeder-out wave.  Compute waves touch
//     only LDS (and load the row characters, 16 rows per 16-byte vector load:
//     an s_load would share lgkmcnt with the LDS traffic and, returning out of
//     order, turn every LDS wait behind it into a wait for it -- 256k: 46.0 ->
//     44.5 ms): every global-memory access of the hand-off sits in a wave of its
//     own, whose stalls stall nobody else.
//   * Hand-off inside the panel: wave w reads wave w-1's last column straight
//     out of w-1's ring; between panels: the feeder-out wave publishes the last
//     compute wave's last column as {tag, value} granules as rows complete, the
//     next panel's feeder-in wave polls them (64 rows per load, the leading run
//     whose tags match) into the feed ring of its first compute wave (nw_dev.h).
//   * No MFMA: integer max/add with no contraction.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nw_dev.h"
#include "nw_internal.h"

namespace nw {
namespace rows {

constexpr int kR = 32;           // ring rows per compute wave (a power of two)
constexpr int kFeedRows = 256;   // feed ring of a panel's first wave (a power of two)
constexpr int kG = 4;            // rows per group (one v_perm word): ring / feed checks, counters
constexpr int kBatch = 8;        // rows per store-wave batch
constexpr int kEnt = 16;         // rows per rowpack entry (16 row characters)
constexpr int kPanelWords = 8;   // per-panel control words (reset with the wave counters)

// Store waves per compute wave.  Under full HBM load one 1 KB store holds its
// wave for ~330 cycles (tools/ubench/panel_store: 4 waves x 1 KB per CU reach
// 6.3 TB/s), so a single store wave serialises those stalls with its own ring
// reads; two or three per ring overlap them.  A workgroup stays <= 16 waves.
constexpr int spw(int nw) { return nw == 4 ? 2 : 3; }

template <int C, int NW>
struct Lay {
    static constexpr int kCols = NW * kWave * C;  // panel width
    static constexpr int kRowB = 4 * kWave * C;   // bytes per ring row
    static constexpr int kRing = kR * kRowB;
    static constexpr int kFeed = NW * kRing;      // byte offset of the feed ring
    static constexpr int kCtl = kFeed + kFeedRows * 4;
    // counters per compute wave w (rows 0 .. v-1 done): [0] written into the
    // ring, [1] (last wave) read by the feeder-out wave, [2] read (left values)
    // by wave w+1, [4 + q] read by its store wave q
    static constexpr int kSPW = spw(NW);
    static constexpr int kCtlWords = 8;
    // panel words: [+0] ticket, [+1] t[0][0], [+2] feed rows in the feed ring
    // (feeder-in), [+3] feed rows read by wave 0
    static constexpr int kPanelWord = NW * kCtlWords;
    static constexpr int kBytes = kCtl + (kPanelWord + kPanelWords) * 4;
    // NW compute waves, NW * kSPW store waves, the feeder-in and feeder-out waves
    static constexpr int kFeedIn = NW * (1 + kSPW);
    static constexpr int kWaves = kFeedIn + 2;
};

static_assert(Lay<4, 4>::kBytes <= 160 * 1024, "ring must fit a CU's LDS");
static_assert(Lay<4, 4>::kWaves <= 16 && Lay<4, 2>::kWaves <= 16 && Lay<4, 1>::kWaves <= 16, "1024 threads");

// Constant address space: uniform loads of the row characters become s_load.
typedef __attribute__((address_space(4))) const uint32_t cu32;

// Inclusive max-scan over the 64 lanes.  update_dpp with INT32_MIN (the max
// identity) as "old" folds into v_max_i32_dpp; lanes with no source keep x.
template <int CTRL, int RM>
__device__ __forceinline__ int32_t scan_step(int32_t x) {
    return max(x, __builtin_amdgcn_update_dpp(INT32_MIN, x, CTRL, RM, 0xF, false));
}
__device__ __forceinline__ int32_t wave_scan_max(int32_t x) {
    x = scan_step<0x111, 0xF>(x);  // row_shr:1
    x = scan_step<0x112, 0xF>(x);  // row_shr:2
    x = scan_step<0x114, 0xF>(x);  // row_shr:4
    x = scan_step<0x118, 0xF>(x);  // row_shr:8
    x = scan_step<0x142, 0xA>(x);  // row_bcast:15 -> rows 1, 3
    x = scan_step<0x143, 0xC>(x);  // row_bcast:31 -> rows 2, 3
    return x;
}

// Substitution score of column k at row q of a 4-row word: PERM: byte q of the
// v_perm result (s' of column k for the 4 mapped row characters); GEN: the
// reference's raw byte compare (serial.cpp:23-24).
template <int MODE>
__device__ __forceinline__ int32_t sub_score(uint32_t pk, uint32_t word, int q, uint32_t a, int32_t msp,
                                             int32_t mmp) {
    if constexpr (MODE == SUB_PERM || MODE == SUB_PERM_SW) {
        return (int32_t)(int8_t)(uint8_t)(pk >> (8 * q));
    } else {
        return ((word >> (8 * q)) & 255u) == a ? msp : mmp;
    }
}

// Compute wave w of panel p: rows 0 .. n2 of its 64*C columns into its ring.
template <int C, int NW, int MODE>
__device__ __forceinline__ void compute_panel(const FillArgs &A, char *__restrict__ lds, int p, int w,
                                              int lane) {
    typedef Lay<C, NW> L;
    constexpr bool SW = is_sw<MODE>();
    constexpr bool PERM = MODE == SUB_PERM || MODE == SUB_PERM_SW;
    const int32_t gap = A.gap;
    const int64_t j0 = A.col0 + (int64_t)p * L::kCols + (int64_t)w * (kWave * C);  // first column of the wave
    const int64_t jl = j0 + (int64_t)C * lane;                                      // of the lane
    int32_t *ctl = (int32_t *)(lds + L::kCtl);
    int32_t *ctr = ctl + w * L::kCtlWords;
    const int32_t nrows = (int32_t)(A.n2 + 1);
    const uint64_t tmo = A.timeout_ticks;
    bool dead = false;

    // ---- row 0: t[0][c] = c*GAP (serial.cpp:16), 0 for SW, or a row band's halo
    // (mpi-horz.cpp:16-40: the previous band's last row, granules carrying this
    // launch's tag, bounded wait).  left0 = t[0][j0-1]; bnd0 = t[0][0].
    int32_t top[C];
#pragma unroll
    for (int k = 0; k < C; ++k) top[k] = SW ? 0 : (int32_t)((jl + k) * (int64_t)gap);
    int32_t left0 = SW ? 0 : (int32_t)((j0 - 1) * (int64_t)gap);
    int32_t bnd0 = 0;
    if (A.halo_in != nullptr) {
        const uint64_t h0 = __builtin_amdgcn_s_memrealtime();
        uint32_t npoll = 0;
        for (;;) {
            bool ok = true;
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const uint64_t g = __hip_atomic_load(A.halo_in + min(jl + k, A.n1), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_SYSTEM);
                top[k] = (int32_t)(uint32_t)g;
                ok &= (uint32_t)(g >> 32) == A.halo_tag;
            }
            const uint64_t gl = __hip_atomic_load(A.halo_in + max(j0 - 1, (int64_t)0), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_SYSTEM);
            const uint64_t g0 = __hip_atomic_load(A.halo_in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            left0 = (int32_t)(uint32_t)gl;
            bnd0 = (int32_t)(uint32_t)g0;
            ok &= (uint32_t)(gl >> 32) == A.halo_tag && (uint32_t)(g0 >> 32) == A.halo_tag;
            if (__all(ok)) break;
            if (++npoll % kPollCheck == 0u) {  // (the error word: not a hot line, nw_dev.h wait_chunk)
                if (ctrl_load(A.ctrl + 1) != 0u) { dead = true; break; }
                if (__builtin_amdgcn_s_memrealtime() - h0 > tmo) {
                    give_up(A.ctrl, 2u, 4, A.halo_in, A.halo_tag, 0);
                    dead = true;
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(4);
        }
    }
    // t[0][0] for the store waves (they store column 0 when col0 = 1); read by
    // them only after this wave's first rows-written counter
    if (w == 0) ctl[L::kPanelWord + 1] = bnd0;

    // ---- x form of row 0 (NW: x = t - GAP*(i+j); SW: x = t - GAP*j; i = 0)
    int32_t x[C];
#pragma unroll
    for (int k = 0; k < C; ++k) x[k] = top[k] - (int32_t)((jl + k) * (int64_t)gap);
    const int32_t xleft0 = j0 >= 1 ? left0 - (int32_t)((j0 - 1) * (int64_t)gap) : kNeg;
    // x[i-1][jl-1] of the next row's column 0 (lane 0: the left neighbour's)
    int32_t cp = __builtin_amdgcn_update_dpp(xleft0, x[C - 1], 0x138 /*wave_shr:1*/, 0xF, 0xF, false);
    // the finals of the current row (what the ring gets); the short-chain form
    // keeps the pre-carry prefixes in x
    int32_t wv[C];
#pragma unroll
    for (int k = 0; k < C; ++k) wv[k] = x[k];

    // ---- per-lane substitution: PERM tables T_k[m] = s(a_k, char m) - off for the
    // mapped row characters m < 8 (7 = in no column: a mismatch); off = 2 GAP
    // (w form) or GAP (SW u form)
    const int32_t off = SW ? gap : 2 * gap;
    const int32_t msp = A.match - off, mmp = A.mismatch - off;
    const uint32_t mmb = ((uint32_t)mmp & 255u) * 0x01010101u;
    uint32_t tlo[C], thi[C], ach[C], mk[C];
    int32_t z[C];  // SW: z_j = -GAP*j, the 0 floor in the u form
#pragma unroll
    for (int k = 0; k < C; ++k) {
        const int64_t c = jl + k;
        const uint32_t a = (c >= 1 && c <= A.n1) ? (uint32_t)A.s1[c - 1] : 0u;
        ach[k] = a;
        z[k] = (int32_t)(-(int64_t)gap * c);
        if constexpr (PERM) {
            const uint32_t m = (c >= 1 && c <= A.n1) ? (uint32_t)A.charmap[a] : 0xFFu;
            mk[k] = m;
            const uint32_t sh = 8u * (m & 3u), keep = ~(255u << sh), put = ((uint32_t)msp & 255u) << sh;
            tlo[k] = m < 4u ? ((mmb & keep) | put) : mmb;
            thi[k] = (m >= 4u && m < 8u) ? ((mmb & keep) | put) : mmb;
        } else {
            tlo[k] = thi[k] = 0u;
        }
    }
    // T_k[m] = max over k' <= k of max(s'(a_k', char m), tfloor): the prefix of
    // the carry's own contributions (see row() below), one v_perm per 4 rows
    const int32_t tfloor = SW ? gap : 0;
    uint32_t ttlo[C], tthi[C];
    {
        int32_t tp[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) tp[m] = INT32_MIN;
#pragma unroll
        for (int k = 0; k < C; ++k) {
            uint32_t lo = 0, hi = 0;
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int32_t sv = PERM ? (mk[k] == (uint32_t)m ? msp : mmp) : 0;
                tp[m] = max(tp[m], max(sv, tfloor));
                const uint32_t b = ((uint32_t)tp[m] & 255u) << (8 * (m & 3));
                if (m < 4) lo |= b; else hi |= b;
            }
            ttlo[k] = lo;
            tthi[k] = hi;
        }
    }

    // ---- the left column, rows 0 .. : x[r][j0-1]
    //   wave w > 0: wave w-1's last column, read out of w-1's ring;
    //   wave 0 of panel > 0 (or a column band's first panel): the feed ring, which
    //     the feeder-in wave fills from the previous panel's granules;
    //   wave 0 of panel 0: the boundary column 0 (x = t[0][0] for NW, 0 for SW),
    //     or nothing when the panels start at column 0 (kNeg).
    // Either way an LDS producer with a rows-available counter.
    enum { SRC_BOUND = 0, SRC_FEED = 1, SRC_RING = 2 };
    const int src = w > 0 ? SRC_RING : p > 0 ? SRC_FEED : SRC_BOUND;
    const int32_t lbound = j0 >= 1 ? (SW ? 0 : bnd0) : kNeg;
    int32_t *feed = (int32_t *)(lds + L::kFeed);
    // byte address of the left value of row r: base + (r & mask) * stride
    const uint32_t lbase = src == SRC_RING ? (uint32_t)((w - 1) * L::kRing + L::kRowB - 4) : (uint32_t)L::kFeed;
    const uint32_t lstride = src == SRC_RING ? (uint32_t)L::kRowB : 4u;
    const uint32_t lmask = src == SRC_RING ? (uint32_t)(kR - 1) : (uint32_t)(kFeedRows - 1);
    const int32_t *prod_written = src == SRC_RING ? ctl + (w - 1) * L::kCtlWords : ctl + L::kPanelWord + 2;
    int32_t *my_consumed = src == SRC_RING ? ctl + (w - 1) * L::kCtlWords + 2 : ctl + L::kPanelWord + 3;

    // ---- the ring: row r of this wave at ring + (r & (kR-1)) * kRowB, lane piece 4C bytes
    const uint32_t rlane = (uint32_t)(w * L::kRing) + (uint32_t)lane * (4u * C);
    // rows computed: whole 64-row trips (the granule slots hold 64 * nblocks rows)
    const int32_t nrow_it = 64 * A.nblocks;
    const int ntrips = A.nblocks;
    uint64_t nslow = 0, wticks = 0, rticks = 0;

    // Ring space: rows 0 .. need-1 must have left the ring (read by my store wave
    // and, for w < NW-1, by wave w+1).  The counters are loaded one group early
    // (cbv) so that the check waits on nothing in the common case.
    // cbr: the counters as loaded (raw: the minimum is taken at the check, so
    // that the loads' latency is not waited for where they are issued)
    int32_t cbr[L::kSPW + 1];
#pragma unroll
    for (int q = 0; q <= L::kSPW; ++q) cbr[q] = 0;
    auto ring_space = [&](int32_t need) {
        int32_t v = cbr[0];
#pragma unroll
        for (int q = 1; q <= L::kSPW; ++q) v = min(v, cbr[q]);
        const int32_t cb = __builtin_amdgcn_readfirstlane(v);
        if (cb < need) {
            const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
            bool d = false;
#pragma unroll
            for (int q = 0; q < L::kSPW; ++q) d |= wait_counter(ctr + 4 + q, need, A.ctrl, 11, tmo) == kDead;
            d |= wait_counter(ctr + (w + 1 < NW ? 2 : 1), need, A.ctrl, 12, tmo) == kDead;
            dead |= d;
            rticks += __builtin_amdgcn_s_memrealtime() - w0;
        }
        lds_order();  // ring writes after the check
    };
    auto ring_poll = [&]() {
#pragma unroll
        for (int q = 0; q < L::kSPW; ++q) cbr[q] = ctr_load(ctr + 4 + q);
        cbr[L::kSPW] = ctr_load(ctr + (w + 1 < NW ? 2 : 1));  // wave w+1 / the feeder-out
    };

    // Left values: the producer (wave w-1 / the feeder-in) must have made rows
    // 0 .. need-1 available (its counter loaded one group early into fbv).
    int32_t fbv = 0;
    auto ring_feed = [&](int32_t need) {
        int32_t fb = __builtin_amdgcn_readfirstlane(fbv);
        if (fb < need) {
            const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
            dead |= wait_counter(prod_written, need, A.ctrl, 14, tmo) == kDead;
            nslow += 1;
            wticks += __builtin_amdgcn_s_memrealtime() - w0;
        }
        lds_order();  // reads after the counter that allowed them
    };
    if (src == SRC_BOUND) {
        for (int i = lane; i < kFeedRows; i += kWave) feed[i] = lbound;  // a constant left column
    }
    // left values of rows [r, r + kG) into lv[] (broadcast ds_read_b32; the kG
    // rows never wrap the ring / feed ring: r is a multiple of kG)
    auto feed_load = [&](int32_t r, int32_t (&lv)[kG]) {
        const uint32_t a = lbase + ((uint32_t)r & lmask) * lstride;
#pragma unroll
        for (int q = 0; q < kG; ++q) lv[q] = *(const int32_t *)(lds + a + (uint32_t)q * lstride);
        if (src != SRC_BOUND) {
            lds_order();
            ctr_store(my_consumed, r + kG);  // (in-order LDS: after the reads)
        }
    };

    // ---- row characters: rowpack16[x + kQOff] = B[x .. x+15], B[y] = s2[y-1]
    // (mapped for PERM): entry e's 16 rows are one 16-byte entry, loaded kWPD
    // entries ahead into wd[e & 3]
    uint32_t wd[4][4];
    // entries (16 rows each) the row characters are loaded ahead (at most 3: a ring of 4)
    constexpr int kWPD = 2;
    static_assert(kWPD >= 1 && kWPD <= 3, "");
    // a VECTOR load (every lane the same 16 bytes: one request), counted on vmcnt:
    // an s_load shares lgkmcnt with the LDS and returns out of order, so every LDS
    // wait issued while it is in flight is an lgkmcnt(0) that also waits for it
    const char *rqv = (const char *)A.rowpack;
    auto wload = [&](int32_t e, uint32_t (&o)[4]) {
        int32_t z = 0;
        asm volatile("" : "+v"(z));  // lane-varying to the compiler: no s_load
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        const v4u v = *(const v4u *)(rqv + ((int64_t)e * kEnt + kQOff) * 16 + z);
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = v[q];
    };

    // ---- one row: x (row r-1) -> x (row r), lv = the left value of row r
    // ---- one row, the short-chain form.  State: P[k] = the previous row's
    // pre-carry prefixes (P[C-1] including its left value) and cp = its carry
    // into this lane (the final value of column jl-1); its finals are
    // max(P[k], cp).  Expanding the recurrence in cp,
    //   m_k = max(W_{k-1} + s_k, W_k) = max(a_k, cp + t_k),
    //   a_k = max(P_{k-1} + s_k, P_k),  t_k = max(s_k, 0)   (NW, w form)
    //   a_k = max(P_{k-1} + s_k, P_k + GAP, z_k), t_k = max(s_k, GAP)   (SW, u form)
    // so the prefix Q_k = max(A_k, cp + T_k) with A, T the prefixes of a, t (T from
    // a v_perm table): only "cp + T, max3 with A and the left value, 6 DPP scan
    // steps, the carry" depend on the previous carry -- 9 dependent operations per
    // row instead of 13.  (The previous row's finals are max(P, cp) because rows
    // are non-decreasing along j in the w / u form, row 0 included.)
    auto row = [&](uint32_t word, const uint32_t (&pks)[C], const uint32_t (&tks)[C], int q, int32_t lv) {
        int32_t Ak[C];
#pragma unroll
        for (int k = 0; k < C; ++k) {
            int32_t a;
            if constexpr (!SW) {
                a = k == 0 ? x[0] : max(x[k - 1] + sub_score<MODE>(pks[k], word, q, ach[k], msp, mmp), x[k]);
            } else {
                const int32_t up = max(x[k] + gap, z[k]);
                a = k == 0 ? up : max(x[k - 1] + sub_score<MODE>(pks[k], word, q, ach[k], msp, mmp), up);
            }
            Ak[k] = k == 0 ? a : max(Ak[k - 1], a);
        }
        int32_t Tk[C];
        if constexpr (PERM) {
#pragma unroll
            for (int k = 0; k < C; ++k) Tk[k] = (int32_t)(int8_t)(uint8_t)(tks[k] >> (8 * q));
        } else {
            const int32_t tfl = SW ? gap : 0;
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const int32_t t = max(sub_score<MODE>(0u, word, q, ach[k], msp, mmp), tfl);
                Tk[k] = k == 0 ? t : max(Tk[k - 1], t);
            }
        }
        const int32_t tot = max(max(Ak[C - 1], cp + Tk[C - 1]), lv);
        const int32_t S = wave_scan_max(tot);
        // exclusive carry: lane l-1's final last column; lane 0: the left value
        const int32_t carry = __builtin_amdgcn_update_dpp(lv, S, 0x138 /*wave_shr:1*/, 0xF, 0xF, false);
        int32_t Q[C];
#pragma unroll
        for (int k = 0; k < C - 1; ++k) Q[k] = max(Ak[k], cp + Tk[k]);
#pragma unroll
        for (int k = 0; k < C - 1; ++k) {
            x[k] = Q[k];                 // pre-carry prefix (state)
            wv[k] = max(Q[k], carry);    // final (ring)
        }
        x[C - 1] = tot;
        wv[C - 1] = S;
        cp = carry;
    };

    // ---- main loop: trips of 64 rows = 16 groups of kG = 4 rows (compile-time
    // group index, so every register ring above is indexed statically).  Row 0
    // (the initial x) goes into the ring without being computed.  The left
    // values of a group are loaded one group ahead.
    int32_t lvA[kG], lvB[kG];
#pragma unroll
    for (int e = 0; e < kWPD; ++e) wload(e, wd[e]);
    if (src != SRC_BOUND) ring_feed(kG);
    feed_load(0, lvA);
    if (src != SRC_BOUND) fbv = ctr_load(prod_written);
    const uint64_t tstart = __builtin_amdgcn_s_memrealtime();
    for (int trip = 0; trip < ntrips && !dead; ++trip) {
        static_for<0, 16>([&](auto gc) {
            constexpr int g = decltype(gc)::value;
            const int32_t r0 = 64 * trip + kG * g;
            int32_t(&lv)[kG] = (g & 1) ? lvB : lvA;
            int32_t(&lvn)[kG] = (g & 1) ? lvA : lvB;
            ring_space(r0 + kG - kR);
            // this group's substitution word (its load was issued kWPD entries ago)
            const uint32_t word = wd[(g >> 2) & 3][g & 3];
            uint32_t pks[C], tks[C];
#pragma unroll
            for (int k = 0; k < C; ++k) {
                pks[k] = PERM ? __builtin_amdgcn_perm(thi[k], tlo[k], word) : 0u;
                tks[k] = PERM ? __builtin_amdgcn_perm(tthi[k], ttlo[k], word) : 0u;
            }
            if constexpr ((g & 3) == 0) wload(r0 / kEnt + kWPD, wd[((g >> 2) + kWPD) & 3]);
            // the next group's left values
            const int32_t rn = r0 + kG;
            if (rn < nrow_it) {
                if (src != SRC_BOUND) ring_feed(rn + kG);
                feed_load(rn, lvn);
            }
#pragma unroll
            for (int u = 0; u < kG; ++u) {
                if (!(g == 0 && u == 0) || trip != 0) row(word, pks, tks, u, lv[u]);
                char *dst = lds + rlane + (uint32_t)((r0 + u) & (kR - 1)) * L::kRowB;
                if constexpr (C == 1) {
                    *(int32_t *)dst = wv[0];
                } else if constexpr (C == 2) {
                    *(int2 *)dst = make_int2(wv[0], wv[1]);
                } else {
                    *(int4 *)dst = make_int4(wv[0], wv[1], wv[2], wv[3]);
                }
                if (u == 1) {
                    // counters for the next group's checks, read mid-group so that
                    // their latency hides behind rows 2 and 3
                    ring_poll();
                    if (src != SRC_BOUND) fbv = ctr_load(prod_written);
                }
            }
            lds_order();
            ctr_store(ctr, r0 + kG);  // rows written
        });
    }
    // every row is in the ring (or the panel is abandoned): release the store
    // waves, the feeder-out and the neighbour waves
    ctr_store(ctr, kDone);
    if (src != SRC_BOUND) ctr_store(my_consumed, kDone);
    if (A.trace != nullptr && lane == 0) {
        uint64_t *tr = A.trace + (int64_t)(p - A.strip0) * kTraceWords;
        if (w == 0) {
            tr[0] = tstart;
            tr[2] = nslow;
            tr[3] = wticks;
            tr[11] = rticks;
        }
        if (w == NW - 1) {
            tr[1] = __builtin_amdgcn_s_memrealtime();
            tr[12] = rticks;
            tr[13] = wticks;
        }
    }
    (void)nrows;
}

// Feeder-in wave of panel p > 0: polls the previous panel's granules (or a
// column band's feed) 64 rows per load and appends the leading run whose tags
// match this launch to the feed ring of compute wave 0, publishing rows
// available in the panel word [+2].  Bounded: gives up (error word) after the
// watchdog interval without progress.
template <int C, int NW>
__device__ __forceinline__ void feeder_in(const FillArgs &A, char *__restrict__ lds, int p, int lane) {
    typedef Lay<C, NW> L;
    if (p == 0) return;  // panel 0's left column is the boundary
    int32_t *ctl = (int32_t *)(lds + L::kCtl);
    int32_t *avail_w = ctl + L::kPanelWord + 2;
    const int32_t *cons = ctl + L::kPanelWord + 3;
    int32_t *feed = (int32_t *)(lds + L::kFeed);
    const bool fed = p == A.strip0 && A.feed_in != nullptr;
    const uint64_t *gin = fed ? A.feed_in : A.gran + (int64_t)((p + A.M - 1) % A.M) * A.gstride;
    const uint32_t tag_in = fed ? A.feed_tag : A.tagbase + (uint32_t)p;
    const int32_t nrow_it = 64 * A.nblocks;
    const uint64_t tmo = A.timeout_ticks;
    int32_t avail = 0, consv = 0;
    uint32_t npoll = 0;
    uint64_t t_last = __builtin_amdgcn_s_memrealtime();
                            // made the 256k fill 44.9 -> 48.7 ms, nw_dev.h wait_chunk)
    while (avail < nrow_it) {
        // feed-ring space for rows avail .. avail+63
        const int32_t need = avail + kWave - kFeedRows;
        if (consv < need) {
            consv = wait_counter(cons, need, A.ctrl, 16, tmo);
            if (consv == kDead) break;
        }
        const int32_t r = avail + lane;
        const uint64_t g = gran_load(gin + min(r, nrow_it - 1));
        const uint64_t ok = __ballot(r < nrow_it && (uint32_t)(g >> 32) == tag_in);
        const int n = ok == ~0ull ? 64 : (int)__builtin_ctzll(~ok);  // leading run
        if (n > 0) {
            if (lane < n) feed[(uint32_t)r & (kFeedRows - 1)] = (int32_t)(uint32_t)g;
            lds_order();
            avail += n;
            ctr_store(avail_w, avail);
            t_last = __builtin_amdgcn_s_memrealtime();
        } else {
            // the error word and the watchdog every kPollCheck empty polls (nw_dev.h wait_chunk)
            if (++npoll % kPollCheck == 0u) {
                if (ctrl_load(A.ctrl + 1) != 0u) break;
                if (__builtin_amdgcn_s_memrealtime() - t_last > tmo) {
                    give_up(A.ctrl, 1u, 13, gin + min(avail, nrow_it - 1), tag_in, (int64_t)(g >> 32));
                    break;
                }
            }
            // (1: sparser polls change nothing here -- the leading panel is store-bound,
            // profiles/r05zc_panel_poll_sleep.txt)
            __builtin_amdgcn_s_sleep(1);
        }
    }
    ctr_store(avail_w, kDone);
}

// Feeder-out wave: publishes the last compute wave's last column, rows 0 .. as
// they complete (up to 32 per store, one {tag, value} granule per row), into
// this panel's granule slot (or a column band's feed, peer memory), and
// releases those ring rows (counter [1] of the last wave).
template <int C, int NW>
__device__ __forceinline__ void feeder_out(const FillArgs &A, char *__restrict__ lds, int p, int lane) {
    typedef Lay<C, NW> L;
    int32_t *ctl = (int32_t *)(lds + L::kCtl);
    int32_t *ctr_l = ctl + (NW - 1) * L::kCtlWords;
    const bool feeds = p == A.strip0 + A.nstrips - 1 && A.feed_out != nullptr;
    uint64_t *gout = feeds ? A.feed_out : A.gran + (int64_t)(p % A.M) * A.gstride;
    const uint64_t tagw = (uint64_t)(feeds ? A.feed_tag : A.tagbase + (uint32_t)p + 1u) << 32;
    const int32_t nrow_it = 64 * A.nblocks;
    const uint32_t lastcol = (uint32_t)((NW - 1) * L::kRing + L::kRowB - 4);
    int32_t pub = 0;
    while (pub < nrow_it) {
        int32_t wr = __builtin_amdgcn_readfirstlane(ctr_load(ctr_l));
        if (wr != kDone && wr <= pub) wr = wait_counter(ctr_l, pub + 1, A.ctrl, 17, A.timeout_ticks);
        if (wr == kDead) break;
        lds_order();
        const int32_t hi = wr == kDone ? nrow_it : min(wr, nrow_it);
        const int32_t n = min(hi - pub, kR);
        uint32_t v = 0;
        if (lane < n) v = *(const uint32_t *)(lds + lastcol + (uint32_t)((pub + lane) & (kR - 1)) * L::kRowB);
        lds_order();
        ctr_store(ctr_l + 1, pub + n);  // ring rows released (in-order LDS: after the reads)
        if (lane < n) gran_store(gout + pub + lane, tagw | v);
        pub += n;
    }
    ctr_store(ctr_l + 1, kDone);
}

// SW: fold a store wave's running maximum into the panel's word A.smax[p].
__device__ __forceinline__ void panel_max(const FillArgs &A, int p, int32_t vmax) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, __shfl_xor(vmax, o));
    if ((threadIdx.x & 63) == 0) atomicMax(A.smax + p, vmax);
}

// Store wave q of compute wave w: its batches of kBatch rows leave the ring, each
// row ONE 256*C-byte row-contiguous segment (lane l: its C columns; C = 4:
// global_store_dwordx4), t = x + GAP*(i+j) (NW) / x + GAP*j (SW).
template <int C, int NW>
__device__ __forceinline__ void store_panel(const FillArgs &A, char *__restrict__ lds, int p, int w, int q,
                                            int lane) {
    typedef Lay<C, NW> L;
    typedef int32_t VT __attribute__((ext_vector_type(C == 1 ? 2 : C)));  // (C = 1 uses .x)
    int32_t *ctl = (int32_t *)(lds + L::kCtl);
    int32_t *ctr = ctl + w * L::kCtlWords;
    const int64_t j0 = A.col0 + (int64_t)p * L::kCols + (int64_t)w * (kWave * C);
    const int64_t jl = j0 + (int64_t)C * lane;
    const int32_t nrows = (int32_t)(A.n2 + 1);
    const bool timing = (A.flags & 1) != 0;
    const int64_t rowb = timing ? 0 : A.pitch * 4;
    char *scr = (char *)(A.scratch + (int64_t)blockIdx.x * kScratchWords);
    const bool sw = A.sw != 0;
    const uint32_t ug = (uint32_t)A.gap;
    uint32_t kc[C];  // GAP * j of the lane's columns (wrapping int32, like the cells)
#pragma unroll
    for (int k = 0; k < C; ++k) kc[k] = ug * (uint32_t)(jl + k);
    const uint32_t ig = sw ? 0u : ug;  // + GAP * i (NW only)
    // store only pieces wholly inside the row (the last panel may overhang the pitch)
    const bool col_ok = jl + C <= A.col_end;
    uint32_t cval = 0;  // SW: columns <= n1
#pragma unroll
    for (int k = 0; k < C; ++k) cval |= (jl + k <= A.n1 ? 1u : 0u) << k;
    int32_t vmax = 0;
    const bool bcol = A.col0 != 0 && p == 0 && w == 0 && !timing && lane == 0;
    const int32_t *bnd0p = ctl + L::kPanelWord + 1;
    int32_t bnd0 = 0;
    char *base = timing ? scr : (char *)(A.table + jl);
    const uint32_t rl = (uint32_t)(w * L::kRing) + (uint32_t)lane * (4u * C);
    int32_t *mine = ctr + 4 + q;
    constexpr int NS = L::kSPW;
    if (A.flags & NW_FLAG_DEBUG_NO_STORE) {  // debug: no store waves (compute-pace probe, timing only)
        ctr_store(mine, kDone);
        return;
    }
    int32_t avail = 0;
    VT v[kBatch];
    int32_t last_lo = -1;  // first row of the batch holding row n2 (halo_out)
    // batches q, q + NS, ... of kBatch rows (round robin over the ring's NS store
    // waves); "read" = every row below the start of my next batch that is mine
    for (int32_t f = q * kBatch; f < nrows; f += NS * kBatch) {
        if (avail < f + kBatch) {
            int32_t sa = __builtin_amdgcn_readfirstlane(ctr_load(ctr));
            if (sa != kDone && sa < f + kBatch) sa = wait_counter(ctr, f + kBatch, A.ctrl, 15, A.timeout_ticks);
            avail = (sa == kDone || sa == kDead) ? INT32_MAX : sa;
            lds_order();
            if (bcol) bnd0 = *bnd0p;
        }
#pragma unroll
        for (int b = 0; b < kBatch; ++b) {
            const char *src = lds + rl + (uint32_t)((f + b) & (kR - 1)) * L::kRowB;
            if constexpr (C == 1)
                v[b].x = *(const int32_t *)src;
            else
                v[b] = *(const VT *)src;
        }
        lds_order();
        ctr_store(mine, f + NS * kBatch);  // release the slots (in-order LDS: after the reads)
#pragma unroll
        for (int b = 0; b < kBatch; ++b) {
            const uint32_t ri = ig * (uint32_t)(f + b);
#pragma unroll
            for (int k = 0; k < C; ++k) v[b][k] = (int32_t)((uint32_t)v[b][k] + kc[k] + ri);
        }
        if (sw) {
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                const bool rok = f + b < nrows;
#pragma unroll
                for (int k = 0; k < C; ++k) vmax = max(vmax, (rok && ((cval >> k) & 1u)) ? v[b][k] : 0);
            }
        }
        char *rp = base + (int64_t)f * rowb;
        if (f + kBatch <= nrows) {
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                if (!col_ok) continue;
                if constexpr (C == 1)
                    *(int32_t *)(rp + b * rowb) = v[b].x;
                else
                    *(VT *)(rp + b * rowb) = v[b];
            }
        } else {
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                if (!col_ok || f + b >= nrows) continue;
                if constexpr (C == 1)
                    *(int32_t *)(rp + b * rowb) = v[b].x;
                else
                    *(VT *)(rp + b * rowb) = v[b];
            }
        }
        if (bcol) {
#pragma unroll
            for (int b = 0; b < kBatch; ++b)
                if (f + b < nrows) *(int32_t *)(rp + b * rowb - 4) = bnd0 + (f + b) * (int32_t)ig;  // column 0
        }
        // Row band: row n2 goes to the next band's halo (system-scope granules,
        // peer HBM over xGMI), straight from the registers that stored it
        if (A.halo_out != nullptr && f + kBatch >= nrows && f < nrows && ctrl_load(A.ctrl + 1) == 0u) {
            const int b = (nrows - 1) - f;
#pragma unroll
            for (int bb = 0; bb < kBatch; ++bb) {
                if (bb != b) continue;
#pragma unroll
                for (int k = 0; k < C; ++k)
                    if (jl + k <= A.n1)
                        __hip_atomic_store(A.halo_out + jl + k, ((uint64_t)A.halo_tag << 32) | (uint32_t)v[bb][k],
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (bcol)
                __hip_atomic_store(A.halo_out, ((uint64_t)A.halo_tag << 32) | (uint32_t)(bnd0 + (int32_t)A.n2 * A.gap),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            last_lo = f;
        }
    }
    (void)last_lo;
    ctr_store(mine, kDone);
    if (sw) panel_max(A, p, vmax);
}

template <int C, int NW, bool SWK>
__global__ __launch_bounds__((64 * Lay<C, NW>::kWaves)) void nw_fill_panels(FillArgs A) {
    typedef Lay<C, NW> L;
    __shared__ __attribute__((aligned(16))) char lds[L::kBytes];
    int32_t *ctl = (int32_t *)(lds + L::kCtl);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // issue priority: the compute waves are the latency-bound chain (their
    // partners on a SIMD are store waves, whose stalls are the memory's)
    if (wave < NW)
        __builtin_amdgcn_s_setprio(2);
    else if (wave >= L::kFeedIn)
        __builtin_amdgcn_s_setprio(1);
    for (;;) {
        if (threadIdx.x == 0) {
            for (int w = 0; w < L::kPanelWord + kPanelWords; ++w) ctl[w] = 0;  // (the panel words too)
            ctl[L::kPanelWord] = (int32_t)atomicAdd(A.ctrl, 1u);
        }
        __syncthreads();
        const int t = __builtin_amdgcn_readfirstlane(ctl[L::kPanelWord]);
        if (t >= A.nstrips) break;
        const int p = A.strip0 + t;
        if (wave < NW) {
            const uint32_t np = __builtin_amdgcn_readfirstlane(ctrl_load(A.nprof));
            const bool perm = A.perm != 0 && np <= kMaxPerm;
            if constexpr (SWK) {
                if (perm)
                    compute_panel<C, NW, SUB_PERM_SW>(A, lds, p, wave, lane);
                else
                    compute_panel<C, NW, SUB_GEN_SW>(A, lds, p, wave, lane);
            } else {
                if (perm)
                    compute_panel<C, NW, SUB_PERM>(A, lds, p, wave, lane);
                else
                    compute_panel<C, NW, SUB_GEN>(A, lds, p, wave, lane);
            }
        } else if (wave < L::kFeedIn) {
            const int b = wave - NW;  // store wave b / NW of ring b % NW
            store_panel<C, NW>(A, lds, p, b % NW, b / NW, lane);
        } else if (wave == L::kFeedIn) {
            feeder_in<C, NW>(A, lds, p, lane);
        } else {
            feeder_out<C, NW>(A, lds, p, lane);
        }
        __syncthreads();  // the rings and counters are reused by the next panel
    }
}

}  // namespace rows

#ifdef NW_ONLY_C
#define NW_PSHAPE(c, nw) ((c) == NW_ONLY_C && (nw) == NW_ONLY_NC)
#else
#define NW_PSHAPE(c, nw) true
#endif

bool panel_shape_ok(int c, int nwaves) {
    switch (c * 16 + nwaves) {
        case 4 * 16 + 4: case 4 * 16 + 2: case 2 * 16 + 4:
        case 4 * 16 + 1: case 2 * 16 + 2: case 1 * 16 + 4:
            return NW_PSHAPE(c, nwaves);
        default:
            return false;
    }
}

int panel_lds_bytes(int c, int nwaves) {
    switch (c * 16 + nwaves) {
        case 4 * 16 + 4: return rows::Lay<4, 4>::kBytes;
        case 4 * 16 + 2: return rows::Lay<4, 2>::kBytes;
        case 2 * 16 + 4: return rows::Lay<2, 4>::kBytes;
        case 4 * 16 + 1: return rows::Lay<4, 1>::kBytes;
        case 2 * 16 + 2: return rows::Lay<2, 2>::kBytes;
        case 1 * 16 + 4: return rows::Lay<1, 4>::kBytes;
        default: return -1;
    }
}

template <int C, int NW>
static void launch_p(const FillArgs &a, int grid, hipStream_t s) {
    const dim3 block(64 * rows::Lay<C, NW>::kWaves);
    if (a.sw)
        hipLaunchKernelGGL((rows::nw_fill_panels<C, NW, true>), dim3(grid), block, 0, s, a);
    else
        hipLaunchKernelGGL((rows::nw_fill_panels<C, NW, false>), dim3(grid), block, 0, s, a);
}

int launch_panels(const FillArgs &a, int c, int nwaves, int grid, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (!panel_shape_ok(c, nwaves)) return (int)hipErrorInvalidValue;
    switch (c * 16 + nwaves) {
#define NW_PCASE(cc, nn) \
        case cc * 16 + nn: if constexpr (NW_PSHAPE(cc, nn)) launch_p<cc, nn>(a, grid, s); break;
        NW_PCASE(4, 4) NW_PCASE(4, 2) NW_PCASE(2, 4)
        NW_PCASE(4, 1) NW_PCASE(2, 2) NW_PCASE(1, 4)
#undef NW_PCASE
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

}  // namespace nw
