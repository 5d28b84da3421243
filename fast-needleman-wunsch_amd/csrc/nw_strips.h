// nw_strips.h -- gfx950 (MI355X) Needleman-Wunsch scoring-table fill: the strip
// kernel (device code; instantiated one shape per TU, nw_strips_<C>x<NC>.hip).
//
// Replaces the fill loops of the reference plugins
//   src/serial/serial.cpp:21-33, src/sentinel/sentinel-mt.cpp:40-62,
//   src/idxarray/idxarray-mt.cpp:43-66
// which all compute, row-major over an int32 table of (n2+1) x (n1+1):
//   t[i][j] = max(t[i-1][j-1] + s(s1[j-1], s2[i-1]), t[i-1][j] + GAP, t[i][j-1] + GAP)
//   t[0][j] = j*GAP, t[i][0] = i*GAP                              (serial.cpp:16-17)
//
// Decomposition (DESIGN.md section 4 has the full picture):
//   * Columns col0 .. n1 are cut into vertical STRIPS of NC*64*C columns (NC
//     chained compute waves of C columns per lane; the tuned shapes are the
//     256-column (4,1), (2,2) and (1,4), csrc/nw_tuned.h -- (2,2) for the SW
//     fill, (4,1) for every row band -- while whole tables as wide as config 3
//     go to the panel kernel, nw_rows.hip; one strip per CU at a time).  col0 = 1 when the table base is
//     laid out so that column 1 starts a 256-byte line (nw_table_offset): then
//     the boundary column 0 (t[i][0] = i*GAP) is not swept at all and an
//     N x N table is exactly N/256 strips.  Each strip is swept top to bottom
//     by one workgroup:
//       - NC COMPUTE waves, wave j owning the strip's columns j*64C .. +64C-1.
//         Lane l owns the C consecutive columns j*64C + C*l + k and at step s
//         computes row i = s - l for all of them -- an anti-diagonal wavefront
//         across the lanes, a left-to-right chain of C cells inside each lane.
//         Cells are held as w = t - GAP*(i+j), in which both gap terms vanish
//         (the store waves add GAP*(i+j) back):
//           d = w_diag + s'(a, b)     v_add_u32_sdwa (a byte of a v_perm result)
//           w = max3(d, w_up, w_left) v_max3_i32
//         s'(a, b) = s(a, b) - 2*GAP comes from a per-lane 8-byte score table
//         indexed by the (mapped) row character: ONE v_perm_b32 gives column
//         k's scores for four consecutive steps.  w_up is the lane's own
//         register; w_left/w_diag of column k > 0 are the lane's own column k-1.
//         Column 0 of the wave takes w_left from lane l-1's column C-1 (DPP
//         wave_shr:1, whose "old" operand feeds lane 0 from the FEED: a ring of
//         the left neighbour's right column in LDS).  Each step's C results go
//         to the wave's LDS ring indexed by ANTI-DIAGONAL (128 slots; slot =
//         step mod 128) with one conflict-free ds_write_b(32*C) at a
//         compile-time offset.  Compute waves issue no table stores: on gfx950
//         a vector store holds its wave for ~45-190 cycles.  A lone wave
//         issues one VALU per ~4 cycles, which is why a strip has several
//         compute waves (one per SIMD) rather than wider lanes.
//       - store waves (kSPR per compute wave): row f of ring j is complete once
//         step f + 63 is written; they read rows back (lane l: slot (f + l)
//         mod 128) and store each as ONE row-contiguous 256*C-byte segment
//         (global_store_dwordx4).  HBM sees only whole, aligned row segments.
//     The waves are coupled by LDS counters (steps written / rows read / feed
//     rows published / iterations done).
//   * Each compute wave reads its right column (lane 63, column C-1) back from
//     its ring 16 rows at a time and publishes it: into the next compute
//     wave's LDS feed ring (+ a counter), or -- for the strip's last wave -- as
//     8-byte {tag, value} granules in HBM (system-scope atomic stores, nw_dev.h
//     NW_GRAN_SCOPE; the data is the flag) for the next strip's first wave, which polls them -- the
//     GPU analogue of idxarray-mt's per-row progress counters
//     (idxarray-mt.cpp:8,44,50-56).
//   * Strips are claimed from an atomic ticket in increasing order by a
//     persistent grid, so a strip's producer is always already running:
//     deadlock-free for any grid size / residency.
//   * Pure int32 VALU + LDS + HBM stores; no MFMA (there is no contraction).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "nw_dev.h"
#include "nw_internal.h"

namespace nw {
constexpr int kR = 128;                // ring slots (anti-diagonals); 64 rows of slack
constexpr int kFeedRows = 256;         // feed ring entries per compute wave

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

// LDS of one workgroup: NC rings of kR anti-diagonal slots (64*C int32 each),
// NC feed rings of kFeedRows int32, the counters.
//   HALF-WORD rings (kHalf, the (2, 4) shape -- 512-column strips, Smith-Waterman
// only): a slot holds the low 16 bits of each cell's w, so that four rings fit in
// 128 KB.  A Smith-Waterman cell satisfies 0 <= t <= max(match, mismatch) *
// min(i, j), so wherever that bound is below 2^16, t = (w + GAP*(i+j)) mod 2^16 is
// exact from the low half alone; the host fixes up the corner where it is not
// (nw_sw.hip nw_sw_fixup) and refuses the shape when that corner is not small.
template <int C, int NC>
struct Lay {
    static constexpr bool kHalf = C == 2 && NC == 4;
    static constexpr int kSlot = (kHalf ? 2 : 4) * kWave * C;  // bytes per ring slot
    static constexpr int kRing = kR * kSlot;          // ring bytes (a power of two)
    static constexpr int kFeed = NC * kRing;          // byte offset of the feed rings
    static constexpr int kCtl = kFeed + NC * kFeedRows * 4;
    // counters, kCtlWords words per compute wave j: [0] steps written, [1] rows of
    // its right column published into wave j+1's feed, [2] iterations done,
    // [3 + q] rows read by its store wave q; then the strip word.  3 + kSPR <= 8
    // are used (the static_assert below); the block is 16 words (64 bytes) since
    // round 5's five store waves, which is padding: 8 would also hold them, but the
    // LDS layout of the measured build is kept as it is
    static constexpr int kCtlWords = 16;
    static constexpr int kStripWord = NC * kCtlWords;
    static constexpr int kBytes = kCtl + (kStripWord + 4) * 4;
    // store waves per compute wave, rows per store-wave batch (kSPR batches in
    // flight <= 64 rows of ring slack)
    // C == 1 rings are GROUPED: a lane keeps 4 steps' results and writes them as
    // one 16-byte record (ds_write_b128 per 4 steps instead of ds_write_b32 per
    // step); group g = step / 4 of the ring holds the 64 lanes' records, lane l
    // at record slot gpos(l) (grp_pos below)
    static constexpr bool kGrp = C == 1;
    // store waves per compute wave: 5 for C = 4 (3 until round 5, 3 / 5 / 7 measured in
    // profiles/r05l_store_waves_ab.txt)
#ifndef NW_SPR22
#define NW_SPR22 2
#endif
    static constexpr int kSPR = C == 4 ? 5 : C == 1 ? 1 : (C == 2 && NC == 2) ? NW_SPR22 : 2;  // ((2,4): 1 / 3 slower, r05t)
    static_assert(3 + kSPR <= kCtlWords, "counter words per compute wave");
    static constexpr int kBatch = C == 4 ? 8 : 16;
    // FEEDER wave (opt-in build NW_FEEDER; one per workgroup, the last): polls the
    // left strip's granules and fills compute wave 0's feed ring + counter (ctl word
    // kFeedWord), so that wave 0 waits on LDS only (it then takes the FEED_LDS path:
    // no granule loads in its prefetch pipeline).  Measured (profiles/
    // r04g_feeder_ab.txt, r05g_feeder_trace.txt, r05zi_feeder_revisited.txt): hop
    // 11.7 -> 7.2-8.5 us on the horizontal band, but the band 32.7 -> 39-42 ms and
    // the SW fill 6.6 -> 7.0 ms: the fed compute waves wait on their feeder at nearly
    // every 16-row chunk (26-28k waits per strip against 5k) and sporadic long hops
    // propagate down the chain ("The feeder question"), so it
    // stays off.  Not for shapes whose workgroup would then exceed 8 waves
    // (register budget).
#ifdef NW_FEEDER
    static constexpr bool kFeeder = NC * (1 + kSPR) < 8;
#else
    static constexpr bool kFeeder = false;
#endif
    static constexpr int kFeedWord = kStripWord + 2;
    static constexpr int kWaves = NC * (1 + kSPR) + (kFeeder ? 1 : 0);
    // compute wave: check ring space every kChk steps, publish progress every kPub
    // (the ring's 64 slots of slack are eaten by these granularities: a batch,
    // the check period plus the staleness of the counter it uses, the publish
    // period -- keep them small)
    static constexpr int kChk = 16;
    static constexpr int kPub = 8;
    // rows per published chunk of the right column (granules / LDS feeds); the code
    // takes 16, 8 or 4.  Finer chunks were slower everywhere (profiles/r05q_gran_ab.txt:
    // horizontal band 30.4-31.4 -> 33.7 (8) / 42.3 ms (4), its hop 11.6 -> 13.7 / 16.5
    // us, SW 64k fill 6.19 -> 7.3 / 9.4 ms): a consumer that finds its prefetched block
    // incomplete pays one poll round trip per chunk, and more chunks per block mean
    // more of them (feed waits per strip 3.4k -> 5.9k / 12.1k)
    static constexpr int kGran = 16;
    static_assert(kGran == 16 || kGran == 8 || kGran == 4, "publish granularity");
};
// Record slot of compute lane a inside a group of a grouped ring: a rotation
// within each 8-lane block, gpos(a) = 8*(a/8) + (a + a/8) % 8.  It keeps both
// sides conflict-free:
//   * ds_write_b128 (lanes served in blocks of 8): gpos % 8 = (a + a/8) % 8 is
//     distinct over a block, so the block covers all 32 banks;
//   * a store wave reads 8 rows x 32 columns per store instruction with
//     ds_read_b32 (two 32-lane halves): half-lane (r, q) (row f+r, r < 4 within
//     the half, q < 8) reads column a = 32h + 4q + k at step f + r + a, bank
//     4 * (gpos(a) % 8) + (f + r + k) % 4; gpos(a) % 8 is distinct over q (a/8
//     steps once per two q while 4q % 8 alternates) and (f + r + k) % 4 over r,
//     so the 32 lanes hit 32 banks.
__device__ __forceinline__ uint32_t grp_pos(uint32_t a) { return (a & ~7u) | ((a + (a >> 3)) & 7u); }

static_assert(Lay<4, 1>::kBytes <= 160 * 1024, "ring must fit a CU's LDS");
static_assert(Lay<2, 2>::kBytes <= 160 * 1024, "ring must fit a CU's LDS");
static_assert(Lay<1, 4>::kBytes <= 160 * 1024, "ring must fit a CU's LDS");

// Rows every store wave of a ring has read out of it (each publishes the
// start of its next batch; all rows below the smallest are out).
template <int NS>
__device__ __forceinline__ int32_t rows_read(const int32_t *rd) {
    int32_t v = ctr_load(rd);
#pragma unroll
    for (int q = 1; q < NS; ++q) v = min(v, ctr_load(rd + q));
    return v;
}
template <int NS>
__device__ __forceinline__ void wait_rows_read(const int32_t *rd, int32_t need, uint32_t *ctrl, uint64_t tmo) {
#pragma unroll
    for (int q = 0; q < NS; ++q) (void)wait_counter(rd + q, need, ctrl, 1, tmo);
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

// How a cell's substitution score is formed.
//   SUB_PERM : the row words hold MAPPED row characters (index 0..7 of the
//              character among s1's distinct ones, 7 = "in no column"); each
//              lane keeps, per column k, the 8-byte table
//              T_k[x] = s(a_k, char x) - 2*GAP (int8).  v_perm_b32(T_k, word)
//              yields column k's scores for the 4 rows of a row word (one
//              byte per step), so per cell d = w_diag + sext(byte): ONE
//              v_add_u32_sdwa, no compare.  Needs <= 7 distinct column
//              characters and both scores - 2*GAP in int8.
//   SUB_UNIT : match - mismatch == 1: d = w_diag + mm' + [a == b]
//              (v_cmp_eq_u32_sdwa -> vcc -> v_addc) on raw characters
//   SUB_GEN  : d = w_diag + (a == b ? ms' : mm')  (v_cmp -> vcc -> v_cndmask, add)
// The compare forms test raw byte equality, the reference's match test
// (serial.cpp:23-24); ms' / mm' / the table bytes have 2*GAP pre-subtracted
// because the cells hold w = t - GAP*(i+j).
//   SUB_PERM_SW / SUB_GEN_SW : Smith-Waterman (local alignment, BASELINE config 5):
//              t = max(0, diag + s, up + GAP, left + GAP) in the same w form as
//              NW, where the 0 floor becomes z = -GAP*(i+j) (run_iter): the
//              substitution exactly as SUB_PERM / SUB_GEN.

template <int QB, int KB, int MODE>
__device__ __forceinline__ int32_t diag_plus_sub(uint32_t w, uint32_t apk, int32_t diag,
                                                 int32_t msp, int32_t mmp) {
    int32_t d;
    if constexpr (MODE == SUB_PERM || MODE == SUB_PERM_SW) {
        // w = v_perm result: byte QB = s'(a_k, row of step QB).  Written in C++ so
        // that the compiler forms the v_add_u32_sdwa (sext BYTE_QB) itself and
        // schedules it: as inline asm it was opaque to the scheduler (C = 4: 99 ->
        // 91 cycles per step, C = 2: 71 -> 64, C = 1: 53 -> 49).
        d = diag + (int32_t)(int8_t)(uint8_t)(w >> (8 * QB));
    } else if constexpr (MODE == SUB_UNIT) {
        asm(
            "v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_%c4 src1_sel:BYTE_%c5\n\t"
            "v_addc_co_u32_e32 %0, vcc, %3, %6, vcc"
            : "=v"(d)
            : "v"(w), "v"(apk), "v"(diag), "i"(QB), "i"(KB), "v"(mmp)
            : "vcc");
    } else {
        int32_t sc;
        asm(
            "v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_%c5 src1_sel:BYTE_%c6\n\t"
            "v_cndmask_b32_e32 %0, %3, %4, vcc"
            : "=v"(sc)
            : "v"(w), "v"(apk), "v"(mmp), "v"(msp), "i"(QB), "i"(KB)
            : "vcc");
        d = diag + sc;
    }
    return d;
}

// Per-lane state of a compute wave on one strip.
template <int C>
struct Lanes {
    int32_t u[C];      // w = t - GAP*(i+j) of the lane's current row, column k
    int32_t z;         // Smith-Waterman: the 0 floor in the w form, -GAP*(i + j) of column 0
    int32_t dg;        // w_diag of column 0 for the next step (= last step's w_left)
    int32_t rr;        // RAMP: row of this lane at the current step
    uint32_t apk;      // raw column characters of the lane, byte k = column k
    uint32_t tlo[C];   // SUB_PERM score tables: bytes 0..3 / 4..7 of T_k
    uint32_t thi[C];
    int32_t cb;        // last value read of the store waves' row counters
    uint32_t rb[2];    // ring byte address of this lane's piece of slot 0 / 64
    uint32_t rc[2];    // read-back address of the right column (see run_iter); grouped
                       // rings: rc[0] = record of lane 63, rc[1] = (lane & 15) - 1
    int32_t rcol;      // right-column value read back, published a few steps later
    uint32_t kcol;     // half-word rings: GAP * (the wave's last column), to rebuild w
    // horizontal-strip band, last strip: the published column is the band's last
    // row, compute lane a* / column k* (FillArgs::tr_pub) instead of lane 63's
    // last column: read back from slot (64*HALF + 16c + pofs) mod kR at pbase
    bool psel;
    int32_t pofs;
    uint32_t pbase;
};

// s_sleep (x 64 clocks) between a waiting compute wave's granule polls in a
// horizontal-strip band (FillArgs::tr; 1 elsewhere).  Every poll is a system-scope
// load of a line its producer is writing through; 255 followers polling every
// ~2 us slowed the band's LEADING strip, which waits for nobody, by 15-17 % (its
// stores share HBM with those polls).  Sleeping 64 x 64 clocks between polls:
// feed waits per strip 3.7k -> 0.7k, leader 29.1 -> 24.6 ms, the band alone
// 30.6 -> 28.4 ms and 2 chained bands 31.3-33.3 -> 30.1-31.0 ms at a hop of 12.3
// instead of 11.5 us (profiles/r05y_poll_sleep.txt).  The vertical sweeps and
// the SW fill, whose chains are latency-bound, lose with it and keep 1.
// (Round 6, with the chain's leader throttled, profiles/r06l_poll_sleep.txt: 1 / 16 /
// 32 / 64 give a mean lag of 9.9 / 10.8 / 11.7 / 12.4 us at a leader of 29.4 / 28.3 /
// 28.1 / 27.0 ms -- so a launch may ask for dense polls, NW_TBAND_DENSE_POLLS.)
constexpr int kPollSleepTr = 64;

// Where a compute wave's feed comes from.
enum FeedSrc { FEED_BOUNDARY = 0, FEED_GRAN = 1, FEED_LDS = 2 };

// The feed of one iteration: the left neighbour's right column (w form) for rows
// 64*it .. 64*it+63, in this wave's LDS feed ring.  `ready` leading chunks of
// kGran rows were found there when the iteration started; before the group that
// first reads chunk c >= ready, run_iter waits for it: FEED_GRAN polls the
// granules (wait_chunk) and writes the kGran values itself, FEED_LDS waits for the
// left compute wave's published-rows counter.
struct Feed {
    int src;             // FeedSrc (uniform)
    const uint64_t *g;   // FEED_GRAN: this lane's granule of the block
    const int32_t *pub;  // FEED_LDS: the left wave's published-rows counter
    int32_t *ring;       // this wave's feed ring (kFeedRows int32)
    uint32_t tag;
    int ready;
    int32_t gap;
    uint32_t nslow;
    uint64_t wticks;
    uint64_t rticks;     // debug trace: time spent waiting for ring space
    bool dead;
    bool trace_pub;      // debug trace: stamp the publish of chunk 0 in this iteration
    uint64_t tpub;
    uint64_t tmo;        // watchdog bound (FillArgs::timeout_ticks)
    bool sparse;         // poll with kPollSleepTr (horizontal strips)
};

// Where a compute wave's right column goes.
struct Out {
    bool off;            // publish nothing (a horizontal band's last strip: its store
                         // waves publish the band's last row, store_strip_tr)
    bool lds;            // into the next compute wave's feed ring (else granules)
    int32_t *ring;       // next wave's feed ring
    int32_t *pub;        // my published-rows counter
    int32_t gap;
};

// 64 wavefront steps of local iteration `it` (steps s = 64*it + u, u < 64) of
// a compute wave.  Step s: compute row s - l on every lane l, write the
// results to ring slot s mod 128 (= 64*HALF + u: a compile-time offset from
// S.rb[HALF]).  Every kPub steps the steps-written counter is published; every
// kChk steps the slots the next kChk overwrite are checked free (rows read by
// the store waves; the counter value was read kChk steps earlier, so its LDS
// latency is hidden).
//   pk   : row words of this iteration (load_packs), 4 x 16 rows
//   b    : block whose right column this iteration publishes (it - 1): rows
//          64b + Gc + i (G = kGran), written by lane 63 at steps 64it + Gc + i - 1,
//          are read back from the ring by lanes i < G after step Gc + G - 2 and
//          published three steps later (the last chunk: after the last step)
//   gp   : this lane's granule of block b (granule output)
//   F    : the feed of this iteration (chunks not yet there are waited for)
template <int C, int NC, int MODE, bool RAMP, int HALF>
__device__ __forceinline__ void run_iter(char *__restrict__ lds, int it, const u32x4 (&pk)[4],
                                         int32_t msp, int32_t mmp, int32_t gap, Lanes<C> &S,
                                         int32_t *ctr, const int32_t *rd, int b, uint64_t *gp,
                                         uint64_t tagw, const Out &O, uint32_t *ctrl, Feed &F,
                                         int lane) {
    typedef typename Vec<C>::T VT;
    typedef Lay<C, NC> L;
    const int4 *feed4 = (const int4 *)(F.ring + ((it & 3) << 6));
    int4 fq = feed4[0];
    const int s0 = it * 64;
    // Ring base of this half.  The barrier keeps LICM from hoisting 64 per-step
    // addresses out of the strip loop (they would stay live in registers); the
    // mask proves the base non-negative, so each step's 64*HALF+u slot offset
    // folds into the ds_write offset field.
    uint32_t rbase = S.rb[HALF];
    asm volatile("" : "+v"(rbase));
    rbase &= 0x3FFFFu;
    char *ringw = lds + rbase;
    int32_t gq[4];  // grouped rings: results of the current 4-step group
    constexpr int G = L::kGran;  // rows per chunk
    constexpr int NCH = 64 / G;  // chunks per block
    // publish chunk c of block b (lanes i < G hold rows 64b + Gc + i)
    auto publish = [&](int c) {
        if (b < 0 || O.off) return;
        if (O.lds) {
            if (lane < G) O.ring[(64 * b + G * c + lane) & (kFeedRows - 1)] = S.rcol;
            lds_order();
            ctr_store(O.pub, 64 * b + G * c + G);
        } else if (lane < G) {
            gran_store(gp + G * c, tagw | (uint32_t)S.rcol);
        }
    };
    static_for<0, 16>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        // ring space for steps s0+4g .. s0+4g+kChk-1: their slots held
        // anti-diagonals s - kR, last needed by row s - kR, so rows
        // <= s0 + 4g + kChk - 1 - kR must have been read
        if constexpr ((4 * g) % L::kChk == 0) {
            const int32_t need = s0 + 4 * g + L::kChk - kR;
            if (__builtin_amdgcn_readfirstlane(S.cb) < need) {
                const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
                wait_rows_read<L::kSPR>(rd, need, ctrl, F.tmo);
                F.rticks += __builtin_amdgcn_s_memrealtime() - w0;  // (trace: ring back-pressure)
            }
            S.cb = rows_read<L::kSPR>(rd);  // for the next check (kChk steps on)
            lds_order();                    // ring writes after the check
        }
        // chunk 4(g+1)/G is read by the feed load below (group g+1 = steps
        // 4g+4 .. 4g+7): wait for it if it was not there when the iteration started
        if constexpr ((4 * (g + 1)) % G == 0 && g + 1 < 16) {
            constexpr int c = 4 * (g + 1) / G;
            if (F.ready <= c) {
                const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
                if (F.src == FEED_GRAN) {
                    const uint64_t v = F.sparse ? wait_chunk<G, kPollSleepTr>(F.g, F.tag, c, ctrl, 2, F.tmo)
                                                : wait_chunk<G, 1>(F.g, F.tag, c, ctrl, 2, F.tmo);
                    F.dead |= !__all(lane / G != c || (uint32_t)(v >> 32) == F.tag);
                    if (lane / G == c) F.ring[((it & 3) << 6) + lane] = (int32_t)(uint32_t)v;
                } else {
                    F.dead |= wait_counter(F.pub, s0 + G * (c + 1), ctrl, 3, F.tmo) == kDead;
                    lds_order();  // feed reads after the counter that published them
                }
                F.nslow += 1;
                F.wticks += __builtin_amdgcn_s_memrealtime() - w0;
                F.ready = c + 1;
            }
        }
        const int4 fcur = fq;
        if constexpr (g + 1 < 16) fq = feed4[g + 1];
        const uint32_t word = pk[g >> 2][g & 3];  // row characters of steps 4g .. 4g+3
        uint32_t sc[C];
        if constexpr (MODE == SUB_PERM || MODE == SUB_PERM_SW) {
#pragma unroll
            for (int k = 0; k < C; ++k) sc[k] = __builtin_amdgcn_perm(S.thi[k], S.tlo[k], word);
        }
        static_for<0, 4>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            constexpr int u = 4 * g + q;
            const int32_t lf = q == 0 ? fcur.x : q == 1 ? fcur.y : q == 2 ? fcur.z : fcur.w;
            int32_t left = __builtin_amdgcn_update_dpp(lf, S.u[C - 1], 0x138 /*wave_shr:1*/,
                                                       0xF, 0xF, false);
            int32_t diag = S.dg;
            S.dg = left;
            // Smith-Waterman: this step's floor -GAP*(i + j) of column 0 (one add per
            // step, off the dependency chain)
            if constexpr (is_sw<MODE>()) S.z -= gap;
            bool act = true;
            if constexpr (RAMP) {
                S.rr += 1;
                asm volatile("" : "+v"(S.rr));  // keep the activity test in the loop
                act = S.rr >= 1;
            }
            VT tv;
            (void)tv;
            static_for<0, C>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                const uint32_t w = (MODE == SUB_PERM || MODE == SUB_PERM_SW) ? sc[k] : word;
                const int32_t d = diag_plus_sub<q, k, MODE>(w, S.apk, diag, msp, mmp);
                int32_t x;
                if constexpr (is_sw<MODE>()) {
                    // t = max(0, t_diag + s, t_up + GAP, t_left + GAP): in the w form
                    // (w = t - GAP*(i+j), as NW) the gap terms vanish and the 0 floor
                    // becomes z = -GAP*(i+j):  w = max3(max(w_diag + s', z), w_up, w_left).
                    // max(w_diag + s', z) does not depend on this step's left value, so
                    // the chain through the row is one v_max3 per cell, as in NW
                    // (v_add, v_max, v_max3 = 3 VALU per cell)
                    const int32_t zk = S.z - gap * k;
                    x = max(max(max(d, zk), S.u[k]), left);
                } else {
                    // w = max(w_diag + s - 2 GAP, w_up, w_left)  (w = t - GAP*(i+j))
                    x = max(max(d, S.u[k]), left);
                }
                diag = S.u[k];
                // lanes still above row 1 hold row 0 (the top boundary / halo)
                if constexpr (RAMP) x = act ? x : S.u[k];
                S.u[k] = x;
                left = x;
                if constexpr (L::kGrp) {
                    gq[u & 3] = x;
                } else {
                    set_comp<C>(tv, k, x);
                }
            });
            if constexpr (L::kHalf) {
                // low halves of the lane's two cells in one dword (v_perm)
                *(uint32_t *)(ringw + u * L::kSlot) =
                    __builtin_amdgcn_perm((uint32_t)tv[1], (uint32_t)tv[0], 0x05040100u);
            } else if constexpr (!L::kGrp) {
                *(VT *)(ringw + u * L::kSlot) = tv;  // ring slot 64*HALF + u
            } else if constexpr ((u & 3) == 3) {
                // group 16*HALF + u/4: this lane's record of steps u-3 .. u
                *(int4 *)(ringw + (u >> 2) * (64 * 16)) = make_int4(gq[0], gq[1], gq[2], gq[3]);
            }
            // right column of block b, chunk c = u / G: read back after the
            // step that completed it (grouped: after its record is written),
            // publish three steps later
            if constexpr (u % G == (L::kGrp ? G - 1 : G - 2)) {
                constexpr int c = u / G;
                uint32_t a;
                if constexpr (L::kGrp) {
                    // lane i < G: step 64*HALF + Gc + i - 1 (mod kR) of lane 63
                    const uint32_t t = (uint32_t)(64 * HALF + G * c + (int)S.rc[1]) & (uint32_t)(kR - 1);
                    a = S.rc[0] + (t >> 2) * (64 * 16) + (t & 3u) * 4u;
                } else {
                    // lane i < G: slot (64*HALF + Gc + i - 1) mod kR, lane 63's last column
                    a = (HALF == 0 && c == 0) ? S.rc[0] : S.rc[1] + (64 * HALF + G * c) * L::kSlot;
                    // (horizontal-strip band: lane a*'s row 64b + Gc + i was written at
                    // step 64it + Gc + i + a* - 64)
                    if (S.psel) a = S.pbase + ((uint32_t)(64 * HALF + G * c + S.pofs) & (uint32_t)(kR - 1)) * L::kSlot;
                }
                if constexpr (L::kHalf) {
                    // lane 63's dword: the wave's last column in its high half; the
                    // cell is t = (w16 + GAP*(i+j)) mod 2^16 (Lay::kHalf), w = t - GAP*(i+j)
                    const uint32_t kc = S.kcol + (uint32_t)gap * (uint32_t)(64 * b + G * c + (lane & (G - 1)));
                    const uint32_t t = ((*(const uint32_t *)(lds + a) >> 16) + kc) & 0xFFFFu;
                    S.rcol = (int32_t)(t - kc);
                } else {
                    S.rcol = *(const int32_t *)(lds + a);
                }
            }
            if constexpr (u % G == (L::kGrp ? 2 : 1) && u > G) {
                publish(u / G - 1);
                if constexpr (u == G + (L::kGrp ? 2 : 1)) {
                    if (F.trace_pub) F.tpub = __builtin_amdgcn_s_memrealtime();
                }
            }
            if constexpr ((u + 1) % L::kPub == 0) {
                lds_order();
                ctr_store(ctr, s0 + u + 1);  // steps written
            }
        });
    });
    publish(NCH - 1);
}

// One strip of a launch: its column strip pk (global: strip0 + k), its place pq
// in the launch's chain of hand-offs (granule slot pq % M, tags tagbase + pq), and
// the row block it belongs to -- a launch may sweep nbl row blocks of equal
// height one after the other (block-cyclic row bands, nw_fill_band_cycle_async):
// each block has its own table, row packs and halo regions.
struct Blk {
    int pk, pq;
    int32_t *table;
    const void *rowpack;
    const uint64_t *halo_in;
    uint64_t *halo_out;
};
__device__ __forceinline__ Blk make_blk(const FillArgs &A, int t) {
    const int blk = A.nbl > 1 ? t / A.nstrips : 0;
    const int k = t - blk * A.nstrips;
    Blk B;
    B.pk = A.strip0 + k;
    B.pq = A.strip0 + t;
    B.table = A.table + (int64_t)blk * A.tstride;
    B.rowpack = (const char *)A.rowpack + (int64_t)blk * A.qstride;
    B.halo_in = (A.halo_in != nullptr && (blk > 0 || A.hin0 != 0)) ? A.halo_in + (int64_t)blk * A.hstride : nullptr;
    B.halo_out = (A.halo_out != nullptr && blk + A.hoshift < A.nbl) ? A.halo_out + (int64_t)(blk + A.hoshift) * A.hstride
                                                                     : nullptr;
    return B;
}

// Compute wave j of strip B.pk.
template <int C, int NC, int MODE, bool TRACE>
__device__ __forceinline__ void compute_strip(const FillArgs &A, char *__restrict__ lds, const Blk &B,
                                              int j, int lane) {
    const int p = B.pk;
    // the debug trace (FillArgs::trace) exists only in the TRACE build of the kernel:
    // its stamps and counters otherwise hold ~20 SGPRs for the whole strip loop
    uint64_t *const trace_p = TRACE ? A.trace : nullptr;
    typedef Lay<C, NC> L;
    constexpr bool SW = is_sw<MODE>();
    const int32_t gap = A.gap;
    // the w form subtracts GAP*(i+j) from every cell (both modes); the top boundary
    // row is t[0][c] = c*GAP for NW, 0 for SW
    const int32_t gw = gap, gt = SW ? 0 : gap;
    const int32_t msp = A.match - 2 * gw, mmp = A.mismatch - 2 * gw;
    const int64_t c0 = A.col0 + (int64_t)p * (NC * 64 * C) + (int64_t)j * (64 * C);
    const int64_t cl = c0 + (int64_t)C * lane;  // first column of this lane
    int32_t *ctr = (int32_t *)(lds + L::kCtl) + j * L::kCtlWords;
    const int32_t *rd = ctr + 3;  // rows read by my store waves
    bool dead = false;
    // Row 0: the boundary t[0][c] = c*GAP (serial.cpp:16), or -- for a row band
    // (mpi-horz.cpp:16-40) -- the previous band's last row, taken from its halo
    // granules once they carry this launch's tag (bounded wait).  bnd0 = t[0][0]
    // (column 0 of the halo for a band), needed when col0 = 1 puts column 0
    // outside the strips.
    int32_t top[C];
    int32_t bnd0 = 0;
#pragma unroll
    for (int k = 0; k < C; ++k) top[k] = (int32_t)((cl + k) * (int64_t)gt);  // SW: row 0 is 0
    if (B.halo_in != nullptr) {
        const uint64_t h0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t n = 1;; ++n) {
            bool ok = true;
#pragma unroll
            for (int k = 0; k < C; ++k) {
                const int64_t c = min(cl + k, A.n1);
                const uint64_t g = __hip_atomic_load(B.halo_in + c, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_SYSTEM);
                top[k] = (int32_t)(uint32_t)g;
                ok &= (uint32_t)(g >> 32) == A.halo_tag;
            }
            const uint64_t g0 = __hip_atomic_load(B.halo_in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            bnd0 = (int32_t)(uint32_t)g0;
            ok &= (uint32_t)(g0 >> 32) == A.halo_tag;
            if (__all(ok)) break;
            if (n % kPollCheck == 0u) {  // (the error word: not a hot line, nw_dev.h wait_chunk)
                if (ctrl_load(A.ctrl + 1) != 0u) { dead = true; break; }
                if (__builtin_amdgcn_s_memrealtime() - h0 > A.timeout_ticks) {
                    give_up(A.ctrl, 2u, 4, B.halo_in, A.halo_tag, 0);
                    dead = true;
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(4);
        }
    }
    // t[0][0] for the store waves (boundary column 0 when col0 = 1); they read it
    // only after this wave's first steps-written counter
    if (j == 0) ((int32_t *)(lds + L::kCtl))[L::kStripWord + 1] = bnd0;
    Lanes<C> S;
    S.apk = 0;
    // SUB_PERM tables: T_k[x] = s(a_k, chars[x]) - 2*GAP for x < 8 (x = 7 and any
    // x >= nprof: a row character in no column, always a mismatch)
    const uint32_t mmb = ((uint32_t)mmp & 255u) * 0x01010101u;
#pragma unroll
    for (int k = 0; k < C; ++k) {
        const int64_t c = cl + k;
        const uint32_t a = (c >= 1 && c <= A.n1) ? (uint32_t)A.s1[c - 1] : 0u;
        S.apk |= a << (8 * k);
        S.u[k] = top[k] - (int32_t)((cl + k) * (int64_t)gw);  // w[0][c] = t[0][c] - GAP*c
        if constexpr (MODE == SUB_PERM || MODE == SUB_PERM_SW) {
            const uint32_t x = (c >= 1 && c <= A.n1) ? (uint32_t)A.charmap[a] : 0xFFu;
            const uint32_t msb = (uint32_t)msp & 255u;
            const uint32_t sh = 8u * (x & 3u), keep = ~(255u << sh), put = msb << sh;
            S.tlo[k] = x < 4u ? ((mmb & keep) | put) : mmb;
            S.thi[k] = (x >= 4u && x < 8u) ? ((mmb & keep) | put) : mmb;
        } else {
            S.tlo[k] = S.thi[k] = 0u;
        }
    }
    S.dg = 0;
    S.rr = -lane - 1;
    // SW floor of column 0 at the step before the first (row rr = -lane - 1)
    S.z = -gap * (int32_t)(-lane - 1 + cl);
    S.cb = 0;
    S.rcol = 0;
    if constexpr (L::kGrp) {
        S.rb[0] = (uint32_t)(j * L::kRing) + grp_pos((uint32_t)lane) * 16u;
    } else {
        S.rb[0] = (uint32_t)(j * L::kRing) + (uint32_t)lane * (uint32_t)(L::kSlot / kWave);
    }
    S.kcol = (uint32_t)gap * (uint32_t)(c0 + 64 * C - 1);
    S.rb[1] = S.rb[0] + 64u * L::kSlot;
    // right-column read-back: lane i < G reads slot (64*HALF + Gc + i - 1) mod kR
    // at lane 63's last column (byte kSlot - 4 of the slot).  rc[1] + offset
    // covers every (HALF, c) but (0, 0), whose lane 0 wraps to slot kR - 1: rc[0].
    if constexpr (L::kGrp) {
        S.rc[0] = (uint32_t)(j * L::kRing) + grp_pos(63u) * 16u;
        S.rc[1] = (uint32_t)((lane & (L::kGran - 1)) - 1);
    } else {
        const int i = lane & (L::kGran - 1);
        S.rc[1] = (uint32_t)(j * L::kRing + i * L::kSlot - 4);  // (i - 1) * kSlot + kSlot - 4
        S.rc[0] = i == 0 ? (uint32_t)(j * L::kRing + L::kRing - 4) : S.rc[1];
    }

    // Feed: the strip's first wave takes the previous strip's right column from
    // its granules (or, for strip 0, the boundary column); later waves take
    // wave j-1's from LDS.  Output: the strip's last wave publishes granules,
    // the others feed wave j+1.
    // a column band's first strip is fed by the left band (feed_in, feed_tag) --
    // also strip 0 of a horizontal-strip row band below the first
    const bool fed = p == A.strip0 && A.feed_in != nullptr;
    Feed F;
    // (with a feeder wave, wave 0's granules arrive through LDS like the later waves' feeds)
    // (debug probe NW_FLAG_DEBUG_NO_CHAIN: every strip unchained -- boundary feed, no publish)
    const bool nochain = (A.flags & NW_FLAG_DEBUG_NO_CHAIN) != 0;
    if (nochain && (A.flags & NW_FLAG_DEBUG_STAGGER)) {  // (probe: the chained sweep's start diagonal)
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t d = (uint64_t)(p - A.strip0) * 1150u;  // 11.5 us per strip (100 MHz ticks)
        while (__builtin_amdgcn_s_memrealtime() - t0 < d) __builtin_amdgcn_s_sleep(8);
    }
    F.src = j > 0 ? FEED_LDS : ((p > 0 || fed) && !nochain) ? (L::kFeeder ? FEED_LDS : FEED_GRAN) : FEED_BOUNDARY;
    F.ring = (int32_t *)(lds + L::kFeed) + j * kFeedRows;
    F.pub = (const int32_t *)(lds + L::kCtl) + (j > 0 ? (j - 1) * L::kCtlWords + 1 : L::kFeeder ? L::kFeedWord : 1);
    const bool feeds = p == A.strip0 + A.nstrips - 1 && A.feed_out != nullptr;
    F.tag = fed ? A.feed_tag : A.tagbase + (uint32_t)B.pq;
    F.gap = gap;
    F.nslow = 0;
    F.wticks = 0;
    F.rticks = 0;
    F.dead = dead;  // (a halo wait may already have given up)
    F.trace_pub = false;
    F.tpub = 0;
    F.tmo = A.timeout_ticks;
    // sparse polls (kPollSleepTr) for the (4, 1) horizontal strips only, unless the
    // launch asks for dense ones (NW_TBAND_DENSE_POLLS: long chains, r06l): the (2, 2)
    // ones poll with them at a 24 us hop, with s_sleep 1 at 11 us (profiles/r06c_tband22.txt)
    F.sparse = A.tr != 0 && NC == 1 && A.tr_dense == 0;
    Out O;
    O.lds = j + 1 < NC;
    O.off = !O.lds && ((A.tr != 0 && feeds && A.tr_store_pub != 0 && (A.flags & 1) == 0) || nochain);
    O.ring = (int32_t *)(lds + L::kFeed) + (j + 1 < NC ? j + 1 : j) * kFeedRows;
    O.pub = ctr + 1;
    O.gap = gap;
    // horizontal-strip band (FillArgs::tr): the band's last row may sit inside
    // the last strip -- publish strip-local column tr_pub (one compute wave)
    S.psel = false;
    S.pofs = 0;
    S.pbase = 0;
    if constexpr (!L::kGrp && NC == 1) {
        if (A.tr != 0 && feeds && !O.off) {
            const int as = A.tr_pub / C, ks = A.tr_pub % C;
            S.psel = true;
            S.pofs = (lane & (L::kGran - 1)) - 64 + as;
            S.pbase = (uint32_t)(as * 4 * C + 4 * ks);
        }
    }
    const int32_t *next_done = ctr + L::kCtlWords + 2;  // iterations done by wave j+1

    const uint64_t *gin = (fed ? A.feed_in : A.gran + (int64_t)((B.pq + A.M - 1) % A.M) * A.gstride) + lane;
    uint64_t *gout = feeds ? A.feed_out : A.gran + (int64_t)(B.pq % A.M) * A.gstride;
    const uint64_t tagw = (uint64_t)(feeds ? A.feed_tag : A.tagbase + (uint32_t)B.pq + 1u) << 32;
    const int nblocks = A.nblocks;
    const int lastb = nblocks - 1;
    uint64_t *gscr = (uint64_t *)(A.scratch + (int64_t)blockIdx.x * kScratchWords) + lane;

    const u32x4 *pkp = (const u32x4 *)B.rowpack;
    // Prefetch pipeline: the row words are loaded PD iterations ahead, the left
    // neighbour's granules (feed) GPD iterations ahead, into NB-deep register
    // rings, so no wait for a load falls inside the steps.  Buffer = iteration
    // mod NB; all loads unconditional (clamped indices).  NB is even so that the
    // ring half (iteration parity) is a function of the buffer index.
    //   The granule distance sets the hand-off's steady state: a consumer whose
    //   prefetch of block b (issued GPD iterations before b) finds it incomplete
    //   takes the slow path, so it settles ~64*GPD steps + the publish lag + a load
    //   latency behind its producer.  But an iteration of a fast shape is shorter
    //   than a loaded load latency, and the wave then stalls on the load it issued
    //   one iteration before.  Measured on one box (profiles/r04e_gpd_ab.txt): GPD =
    //   1 cuts the (4,1) horizontal band's hop 18.2 -> 11.7 us (band 32.7 -> 31.7
    //   ms) but slows the (2,2) SW 64k fill 6.2 -> 7.4 ms (GPD = 2: no change,
    //   profiles/r04h_step_loop_gpd2.txt); so (4,1) -- the horizontal strips' shape
    //   -- uses 1, the others 3 (the row words' distance).
    constexpr int NB = 4, PD = NB - 1;
    constexpr int GPD = (C == 4 && NC == 1) ? 1 : 3;
    static_assert(GPD >= 1 && GPD <= PD, "granule prefetch distance");
    uint64_t gb[NB];
    u32x4 pkb[NB][4];
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        if (!L::kFeeder && i < GPD) gb[i] = gran_load(gin + (int64_t)min(i, lastb) * 64);  // block i, for iteration i
        load_packs(pkp, i, lane, pkb[i]);
    }

    const uint64_t tstart = __builtin_amdgcn_s_memrealtime();
    const uint64_t cstart = __builtin_amdgcn_s_memtime();
    uint64_t tq1 = 0, tmid = 0;  // trace: times iterations nblocks/4 and nblocks/2 started
    uint64_t tsee = 0, twait = 0;  // trace: see / wait start, block nblocks/2 chunk 0
    uint64_t tin = 0;              // trace: shader cycles spent inside run_iter

    // Iteration it: feed for block it (consumes buffer it % NB), prefetch for
    // it+PD, 64 steps, block it-1's right column published.  A watchdog trip
    // marks the strip dead; it is abandoned at the boundary.
    auto iter = [&](int it, auto cons_c, auto ramp_c) {
        constexpr int CONS = decltype(cons_c)::value;  // it % NB
        constexpr int ISS = (CONS + PD) % NB;          // (it + PD) % NB
        constexpr int GISS = (CONS + GPD) % NB;        // (it + GPD) % NB
        constexpr int HALF = CONS & 1;                 // it % 2
        constexpr bool RAMP = decltype(ramp_c)::value;
        const bool traced = trace_p != nullptr && it == nblocks / 2;
        if (trace_p != nullptr) {
            if (it == nblocks / 4) tq1 = __builtin_amdgcn_s_memrealtime();
            if (traced) tmid = __builtin_amdgcn_s_memrealtime();
            F.trace_pub = it == nblocks / 2 + 1;
        }
        // feed-ring space for this iteration's publish (rows of block it-1 land
        // where rows of block it-5 were): wave j+1 must have finished it-5
        if (O.lds && it >= 5) F.dead |= wait_counter(next_done, it - 4, A.ctrl, 5, A.timeout_ticks) == kDead;
        constexpr int G = L::kGran;
        F.ready = 64 / G;
        if (it < nblocks) {
            if (F.src == FEED_GRAN) {
                uint64_t gv = gb[CONS];  // block it, loaded PD iterations ago
                F.g = gin + (int64_t)it * 64;
                F.ready = chunks_ready<G>(gv, F.tag);
                if (F.ready == 0) {  // chunk 0 is needed right away
                    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
                    if (traced) twait = w0;
                    gv = F.sparse ? wait_chunk<G, kPollSleepTr>(F.g, F.tag, 0, A.ctrl, 6, A.timeout_ticks)
                                  : wait_chunk<G, 1>(F.g, F.tag, 0, A.ctrl, 6, A.timeout_ticks);
                    F.dead |= !__all(lane >= G || (uint32_t)(gv >> 32) == F.tag);
                    F.nslow += 1;
                    F.wticks += __builtin_amdgcn_s_memrealtime() - w0;
                    F.ready = max(1, chunks_ready<G>(gv, F.tag));
                }
                F.ring[((it & 3) << 6) + lane] = (int32_t)(uint32_t)gv;
            } else if (F.src == FEED_LDS) {
                int32_t pv = __builtin_amdgcn_readfirstlane(ctr_load(F.pub));
                if (pv < it * 64 + G) {
                    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
                    if (traced) twait = w0;
                    pv = wait_counter(F.pub, it * 64 + G, A.ctrl, 7, A.timeout_ticks);
                    F.dead |= pv == kDead;
                    F.nslow += 1;
                    F.wticks += __builtin_amdgcn_s_memrealtime() - w0;
                }
                F.ready = min(64 / G, (pv - it * 64) / G);
                lds_order();  // feed reads after the counter that published them
            } else {
                // the unfed leader of a horizontal band sleeps a little per iteration
                // (FillArgs::lead_sleep), so that a follower that runs slower for a
                // while keeps up instead of delaying every strip below it
                for (int z = 0; z < A.lead_sleep; ++z) __builtin_amdgcn_s_sleep(1);
                // strip 0, wave 0: left of column col0 is the boundary column:
                // w[r][0] = t[r][0] - GAP*r = t[0][0] with col0 = 1, "minus infinity"
                // when col0 = 0 (the lane holding column 0 then computes
                // w[r][0] = w[r-1][0], i.e. t[r][0] = t[r-1][0] + GAP)
                // (SW: t[r][0] = 0, w[r][0] = -GAP*r)
                F.ring[((it & 3) << 6) + lane] = SW && A.col0 ? -gap * (64 * it + lane) : A.col0 ? bnd0 : kNeg;
            }
            if (traced) tsee = __builtin_amdgcn_s_memrealtime();
        } else if (F.src != FEED_LDS) {
            // past the last block: every lane's row is beyond n2
            F.ring[((it & 3) << 6) + lane] = kNeg;
        }
        if constexpr (!L::kFeeder) gb[GISS] = gran_load(gin + (int64_t)min(it + GPD, lastb) * 64);
        load_packs(pkp, it + PD, lane, pkb[ISS]);
        const int b = it - 1;  // block whose right column this iteration publishes
        uint64_t *gp = (b >= 0 && b < nblocks) ? gout + (int64_t)b * 64 + lane : gscr;
        const uint64_t ti0 = trace_p != nullptr ? __builtin_amdgcn_s_memtime() : 0;
        run_iter<C, NC, MODE, RAMP, HALF>(lds, it, pkb[CONS], msp, mmp, gap, S, ctr, rd, b, gp, tagw,
                                          O, A.ctrl, F, lane);
        if (trace_p != nullptr) tin += __builtin_amdgcn_s_memtime() - ti0;
        ctr_store(ctr + 2, it + 1);  // iterations done (feed-ring space for wave j-1)
        dead = F.dead;
    };
    // iteration 0 ramps the wavefront in (lanes above row 1 hold row 0); row
    // 64*nblocks - 1 completes (lane 63) at step 64*nblocks + 62, iteration nblocks
    const int nit = nblocks + 1;
    iter(0, std::integral_constant<int, 0>{}, std::true_type{});
    for (int it = 1; it < nit && !dead; it += NB) {
        iter(it, std::integral_constant<int, 1>{}, std::false_type{});
        if (it + 1 >= nit || dead) break;
        iter(it + 1, std::integral_constant<int, 2>{}, std::false_type{});
        if (it + 2 >= nit || dead) break;
        iter(it + 2, std::integral_constant<int, 3>{}, std::false_type{});
        if (it + 3 >= nit || dead) break;
        iter(it + 3, std::integral_constant<int, 0>{}, std::false_type{});
    }
    // every row is in the ring (or the strip is abandoned): release the store
    // waves and the compute waves waiting on me
    ctr_store(ctr, kDone);
    ctr_store(ctr + 1, kDone);
    ctr_store(ctr + 2, kDone);
    if (trace_p != nullptr && lane == 0) {
        uint64_t *tr = trace_p + (int64_t)(B.pq - A.strip0) * kTraceWords;
        if (j == 0) {
            tr[0] = tstart;
            tr[2] = F.nslow;
            tr[3] = F.wticks;
            tr[4] = tq1;
            tr[5] = tmid;
            tr[6] = cstart;  // shader clock (s_memtime)
            tr[9] = tsee;
            tr[10] = twait;
            tr[11] = F.rticks;
            tr[14] = tin;
        }
        if (j == NC - 1) {
            tr[1] = __builtin_amdgcn_s_memrealtime();
            tr[7] = __builtin_amdgcn_s_memtime();
            tr[8] = F.tpub;
            tr[12] = F.rticks;
            tr[13] = F.wticks;
            tr[15] = tin;
        }
    }
}

// Feeder wave of strip B.pk (Lay::kFeeder): the left neighbour's right column
// arrives as {tag, value} granules in 64-row blocks (its last compute wave, or a
// feed_in of the band / column band to the left, publishes them); this wave polls
// them -- one 64-granule load, the leading run of rows carrying the tag goes into
// compute wave 0's feed ring (row r at r mod kFeedRows) and the rows-available
// counter ctl[kFeedWord] -- so that wave 0's prefetch pipeline holds no granule
// loads and its waits are LDS waits.  Ring space: row r overwrites row r - 256,
// read by wave 0's iteration (r - 256) / 64, so the wave waits for wave 0's
// iterations-done counter.  Serial polls (nw_dev.h wait_chunk): one load in flight.
template <int C, int NC, bool TRACE>
__device__ __forceinline__ void feed_strip(const FillArgs &A, char *__restrict__ lds, const Blk &B, int lane) {
    typedef Lay<C, NC> L;
    int32_t *ctl = (int32_t *)(lds + L::kCtl);
    int32_t *avail_w = ctl + L::kFeedWord;
    const int p = B.pk;
    const bool fed = p == A.strip0 && A.feed_in != nullptr;
    if (!(p > 0 || fed)) return;  // wave 0 takes the boundary column
    const int32_t *done0 = ctl + 2;  // compute wave 0: iterations done
    int32_t *ring = (int32_t *)(lds + L::kFeed);
    const uint64_t *gin = fed ? A.feed_in : A.gran + (int64_t)((B.pq + A.M - 1) % A.M) * A.gstride;
    const uint32_t tag = fed ? A.feed_tag : A.tagbase + (uint32_t)B.pq;
    const int32_t nrow = 64 * A.nblocks;
    const uint64_t tmo = A.timeout_ticks;
    int32_t avail = 0, consv = 0;
    uint64_t t_last = __builtin_amdgcn_s_memrealtime();
    uint32_t idle = 0;
    // debug trace (words 19..23): ring-space wait total, the longest no-data streak,
    // the row it waited for, when it ended, number of streaks over 100 us
    const bool traced = TRACE && A.trace != nullptr;
    uint64_t t_ring = 0, t_max = 0, t_max_end = 0, n_long = 0;
    int32_t r_max = 0;
    while (avail < nrow) {
        const int32_t need = ((avail + 63) >> 6) - 3;  // iterations wave 0 must have finished
        if (consv < need) {
            const uint64_t w0 = traced ? __builtin_amdgcn_s_memrealtime() : 0;
            consv = wait_counter(done0, need, A.ctrl, 21, tmo);
            if (traced) t_ring += __builtin_amdgcn_s_memrealtime() - w0;
            if (consv == kDead) break;
        }
        const int32_t r = avail + lane;
        const uint64_t g = gran_load(gin + min(r, nrow - 1));
        const uint64_t ok = __ballot(r < nrow && (uint32_t)(g >> 32) == tag);
        const int n = ok == ~0ull ? 64 : (int)__builtin_ctzll(~ok);  // leading run
        if (n > 0) {
            if (lane < n) ring[(uint32_t)r & (kFeedRows - 1)] = (int32_t)(uint32_t)g;
            lds_order();
            avail += n;
            ctr_store(avail_w, avail);
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            if (traced && idle > 0) {
                const uint64_t streak = now - t_last;
                if (streak > t_max) {
                    t_max = streak;
                    r_max = avail - n;
                    t_max_end = now;
                }
                n_long += streak > 10000u ? 1u : 0u;  // > 100 us
            }
            t_last = now;
            idle = 0;
        } else {
            // the error word and the watchdog every 32 empty polls only: every idle
            // feeder of the chip re-reading the one error word after each poll is a
            // hot line (as a scalar poll of it from every wave is, nw_dev.h)
            if ((++idle & 31u) == 0u) {
                if (ctrl_load(A.ctrl + 1) != 0u) break;
                // twice the bound: a wait of the strip's own compute waves (its halo) or
                // of the producer upstream is the root cause and must be the one to report
                if (__builtin_amdgcn_s_memrealtime() - t_last > 2 * tmo) {
                    give_up(A.ctrl, 1u, 22, gin + min(avail, nrow - 1), tag, (int64_t)(g >> 32));
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    ctr_store(avail_w, kDone);  // (also releases wave 0 when the wait gave up: the error word is set)
    if (traced && lane == 0) {
        uint64_t *tr = A.trace + (int64_t)(B.pq - A.strip0) * kTraceWords;
        tr[19] = t_ring;
        tr[20] = t_max;
        tr[21] = (uint64_t)r_max;
        tr[22] = t_max_end;
        tr[23] = n_long;
    }
}

// Smith-Waterman: fold a store wave's running maximum into the strip's word
// A.smax[p] (zeroed before the launch; the locate kernel reads them).
__device__ __forceinline__ void strip_max(const FillArgs &A, int p, int32_t vmax) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) vmax = max(vmax, __shfl_xor(vmax, off));
    if ((threadIdx.x & 63) == 0) atomicMax(A.smax + p, vmax);
}

// Store wave q of compute wave j on strip p: rows 0 .. n2 of ring j leave as
// whole row segments.  One 16-byte-per-lane store covers NR = 4/C rows (1 KB:
// a row of a C = 4 ring, two rows of a C = 2 ring): lane l takes row
// f + l / (16C), columns 4 * (l % (16C)) .. +3, i.e. the pieces of the NR
// compute lanes a = NR * (l % (16C)) + m that wrote them, each in slot
// (row + a) mod kR.  Rows go in batches of kBatch, dealt round robin to the
// kSPR store waves of the ring: wait until the compute wave has written the
// batch, read it from the ring, store it, then release its slots.  Under full
// HBM load one store instruction holds its wave for ~190 cycles, which is why
// one compute wave has several store waves.
template <int C, int NC>
__device__ __forceinline__ void store_strip(const FillArgs &A, char *__restrict__ lds, const Blk &B,
                                            int j, int q, int lane) {
    const int p = B.pk;
    typedef typename Vec<C>::T VT;
    typedef Lay<C, NC> L;
    constexpr int NR = 4 / C;                  // rows per store instruction
    constexpr int Q = 16 * C;                  // lanes per row
    constexpr int BATCH = L::kBatch;
    constexpr int NS = L::kSPR;
    constexpr int NG = BATCH / NR;             // stores per batch
    constexpr uint32_t kMask = (uint32_t)L::kRing - 1u;
    int32_t *ctr = (int32_t *)(lds + L::kCtl) + j * L::kCtlWords;
    const char *ring = lds + j * L::kRing;
    const int64_t c0 = A.col0 + (int64_t)p * (NC * 64 * C) + (int64_t)j * (64 * C);
    const int32_t nrows = (int32_t)(A.n2 + 1);
    const bool timing = (A.flags & 1) != 0;
    const int ro = lane / Q, cq = lane % Q;
    // the last strip may overhang the pitch: store only 16-byte pieces that lie
    // wholly inside the row (with col0 = 1 a piece straddling the pitch would
    // reach the next row's column 0; nw_table_pitch leaves room for column n1)
    const bool col_ok = c0 + 4 * cq + 4 <= A.col_end;
    const int64_t rowb = timing ? 0 : A.pitch * 4;
    char *scr = (char *)(A.scratch + (int64_t)blockIdx.x * kScratchWords);
    const int32_t f0 = q * BATCH;
    // the ring holds w = t - GAP*(r + c) (run_iter): kc[e] = GAP*(r + c) of element
    // e of this lane's piece in its current batch (wrapping int32, like the cells);
    const uint32_t ug = (uint32_t)A.gap;  // (both modes: the w form)
    uint32_t kc[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) kc[e] = ug * (uint32_t)(f0 + ro) + ug * (uint32_t)(c0 + 4 * cq + e);
    // SW: running maximum of this lane's cells (columns <= n1 only) for the
    // strip's best-cell word A.smax[p]
    uint32_t cval = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) cval |= (c0 + 4 * cq + e <= A.n1 ? 1u : 0u) << e;
    int32_t vmax = 0;
    char *rowp = timing ? scr : (char *)(B.table + c0) + (int64_t)f0 * rowb;
    const uint32_t voff = (uint32_t)(ro * rowb) + (uint32_t)cq * 16u;
    // col0 = 1: strip 0's first ring also stores the boundary column 0,
    // t[r][0] = t[0][0] + r*GAP (t[0][0] = 0, or the halo's column 0 for a band)
    const bool bcol = A.col0 != 0 && p == 0 && j == 0 && !timing;
    int32_t bnd0 = 0;  // t[0][0]: from compute wave 0 (after its halo wait), read below
    const int32_t *bnd0p = (const int32_t *)(lds + L::kCtl) + L::kStripWord + 1;
    uint32_t pa[NR];  // ring byte address of piece m of this lane's row
#pragma unroll
    for (int m = 0; m < NR; ++m) {
        const int a = NR * cq + m;
        pa[m] = (uint32_t)((f0 + ro + a) % kR) * L::kSlot + (uint32_t)a * (uint32_t)(L::kSlot / kWave);
    }
    // `rows` further down the ring (the piece offset a * 4C < kSlot survives the mask)
    auto adv = [&](uint32_t x, uint32_t rows) { return (x + rows * L::kSlot) & kMask; };
    int32_t *mine = ctr + 3 + q;
    if (A.flags & NW_FLAG_DEBUG_NO_STORE) {  // debug: no store waves at all (compute-pace probe, timing only)
        ctr_store(mine, kDone);
        return;
    }
    int32_t avail = 0;  // rows complete in the ring (steps written - 63)
    for (int32_t f = f0; f < nrows; f += NS * BATCH) {
        const int32_t want = min(f + BATCH, nrows);
        if (avail < want) {
            int32_t sa = __builtin_amdgcn_readfirstlane(ctr_load(ctr));
            if (sa != kDone && sa - 63 < want) sa = wait_counter(ctr, want + 63, A.ctrl, 8, A.timeout_ticks);
            avail = (sa == kDone || sa == kDead) ? nrows : min(sa - 63, nrows);
            lds_order();  // ring reads after the counter that released them
            if (bcol) bnd0 = *bnd0p;
        }
        if (A.flags & NW_FLAG_DEBUG_DRAIN) {  // debug: drain the ring without reading it (compute-pace probe)
            rowp += NS * BATCH * rowb;
            lds_order();
            ctr_store(mine, f + NS * BATCH);
            continue;
        }
        u32x4 v[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
#pragma unroll
            for (int m = 0; m < NR; ++m) {
                if constexpr (L::kHalf) {
                    // two cells' low halves: t = (w16 + GAP*(i+j)) mod 2^16 (Lay::kHalf)
                    const uint32_t x = *(const uint32_t *)(ring + pa[m]);
                    pa[m] = adv(pa[m], NR);
#pragma unroll
                    for (int k = 0; k < C; ++k)
                        v[g][m * C + k] = (((k == 0 ? x : x >> 16) + kc[m * C + k] + ug * (uint32_t)(g * NR)) & 0xFFFFu);
                } else {
                    const VT x = *(const VT *)(ring + pa[m]);
                    pa[m] = adv(pa[m], NR);
#pragma unroll
                    for (int k = 0; k < C; ++k)
                        v[g][m * C + k] = (uint32_t)comp<C>(x, k) + kc[m * C + k] + ug * (uint32_t)(g * NR);
                }
            }
        }
#pragma unroll
        for (int m = 0; m < NR; ++m) pa[m] = adv(pa[m], (NS - 1) * BATCH);  // skip the others'
#pragma unroll
        for (int e = 0; e < 4; ++e) kc[e] += ug * (uint32_t)(NS * BATCH);
        // the batch is in registers: release its ring slots before the stores
        // (in-order LDS: the counter is written after the reads have read)
        lds_order();
        ctr_store(mine, f + NS * BATCH);
        if (A.sw) {
            if (want - f == BATCH && cval == 0xFu) {  // interior batch: every cell counts
#pragma unroll
                for (int g = 0; g < NG; ++g)
#pragma unroll
                    for (int e = 0; e < 4; ++e) vmax = max(vmax, (int32_t)v[g][e]);
            } else {
#pragma unroll
                for (int g = 0; g < NG; ++g) {
                    const bool rok = f + g * NR + ro < nrows;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        vmax = max(vmax, (rok && ((cval >> e) & 1u)) ? (int32_t)v[g][e] : 0);
                }
            }
        }
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
        if (bcol) {
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                const int32_t r = f + g * NR + ro;
                if (cq == 0 && r < nrows)
                    *(int32_t *)(rowp + (int64_t)g * NR * rowb + (int64_t)voff - 4) = bnd0 + r * (A.sw ? 0 : (int32_t)ug);
            }
        }
        rowp += NS * BATCH * rowb;
    }
    ctr_store(mine, kDone);
    if (A.sw) strip_max(A, p, vmax);
    // Row band: hand this ring's columns of the last row (n2) to the next band.
    // The table stores are plain (write-back L2), so: drain them, write the XCD's
    // L2 back (agent release), re-read the row with sc1 loads, publish
    // system-scope granules (write-through; peer HBM over xGMI when the next
    // band lives on another GPU).  (The store wave that stored row n2 does it.)
    if (B.halo_out != nullptr && ((nrows - 1) / BATCH) % NS == q && ctrl_load(A.ctrl + 1) == 0u) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const int32_t *last = B.table + A.n2 * A.pitch;
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const int64_t c = c0 + (int64_t)C * lane + k;
            if (c <= A.n1) {
                const uint32_t x = (uint32_t)__hip_atomic_load(last + c, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(B.halo_out + c, ((uint64_t)A.halo_tag << 32) | x,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        if (bcol && lane == 0)
            __hip_atomic_store(B.halo_out,
                               ((uint64_t)A.halo_tag << 32) | (uint32_t)(bnd0 + (int32_t)A.n2 * A.gap),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Store wave q of ring j of a HORIZONTAL strip (row band in horizontal strips,
// nw_fill_tband_async; the (4, 1) and (2, 2) shapes).  The strip runs along the
// band's rows: ring row x (step s holds rows x = s - a of compute lanes a) is table
// COLUMN x, and compute lane a of wave j holds table rows y = c0 + C a + k, k < C
// (c0 = the strip's first global row + 64 C j; local row y - tr_y0).  Columns leave
// in batches of 32 (x = 1 + 32b .. +31: 128-byte row segments, aligned when column
// 1 starts a 256-byte line), dealt round robin to the ring's kSPR store waves.  Store
// lane (g, l8) = (lane / 8, lane % 8) takes, for each block of 8 compute lanes
// a = 8 blk + l8, the C x 4 tile rows C a .. C a + C-1 x columns x0 + 4g .. +3 with
// four ds_read_b(32 C) (slot (x + a) mod kR, byte 4 C a: the 8 lanes the LDS serves
// together hit 8 distinct pieces of one slot) and stores it as C 16-byte row pieces:
// one store instruction = 8 rows (stride C) x 128 bytes.  A wave publishes its first
// batch start before reading anything (rows below it are none of its business): with
// 3 waves x 32 columns the ring's slack would otherwise run out before the third
// wave's first batch is complete.
template <int C, int NC>
__device__ __forceinline__ void store_strip_tr(const FillArgs &A, char *__restrict__ lds, const Blk &B,
                                               int j, int q, int lane) {
    static_assert((C == 4 && NC == 1) || (C == 2 && NC == 2), "horizontal strips: the (4, 1) / (2, 2) shapes");
    typedef Lay<C, NC> L;
    typedef typename Vec<C>::T VT;
    constexpr int BATCH = 32, NS = L::kSPR, NBLK = 8;
    static_assert(BATCH + 63 + L::kChk + L::kPub <= kR, "a batch must fit the ring's slack");
    const int p = B.pk;
    int32_t *ctr = (int32_t *)(lds + L::kCtl) + j * L::kCtlWords;
    const char *ring = lds + j * L::kRing;
    // global row of ring j's compute lane 0's first piece
    const int64_t c0 = A.col0 + (int64_t)p * (64 * C * NC) + (int64_t)j * (64 * C);
    const int32_t nx = (int32_t)(A.n2 + 1);             // ring rows = table columns 0 .. n2
    const bool timing = (A.flags & 1) != 0;
    const int g = lane >> 3, l8 = lane & 7;
    const uint32_t ug = (uint32_t)A.gap;
    int32_t *mine = ctr + 3 + q;
    const int32_t f0 = 1 + q * BATCH;
    ctr_store(mine, f0);
    if (A.flags & NW_FLAG_DEBUG_NO_STORE) {  // debug: no store waves (compute-pace probe, timing only)
        ctr_store(mine, kDone);
        return;
    }
    // The band's last strip publishes the band's last row (strip-local row tr_pub =
    // 64 C j* + C a* + k*: ring j*, compute lane a*, piece element k*) into the next
    // band's feed, one {tag, w} granule per column, from HERE rather than from the
    // compute wave: the feed is fine-grained memory whose system-scope stores complete
    // slowly, and a compute wave that issued them waits for them at each of its own
    // prefetch waits (vmcnt counts stores too).  The 8 lanes (g, a* % 8) of ring j*'s
    // store waves hold the row's 32 columns of each batch (block a* / 8, element k*).
    // Store wave 0 of ring j* also publishes column 0 (w = t - GAP*y = 0 for the
    // boundary column t[y][0] = y*GAP) and the padding granules of the last 64-column
    // block (tag only).
    const int jpub = A.tr_pub / (64 * C), lpub = A.tr_pub % (64 * C);
    const bool tpub = A.tr != 0 && A.tr_store_pub != 0 && A.feed_out != nullptr &&
                      p == A.strip0 + A.nstrips - 1 && !timing && j == jpub;
    const int pas = lpub / C, pks = lpub % C;
    const bool plane = tpub && l8 == (pas & 7);
    const uint64_t ptag = (uint64_t)A.feed_tag << 32;
    if (tpub && q == 0) {
        const int32_t x = lane == 0 ? 0 : nx - 1 + lane;
        if (x < 64 * A.nblocks) gran_store(A.feed_out + x, ptag);
    }
    // rows of this lane: y = c0 + C (8 blk + l8) + k; valid while y <= n1 (the band's last row)
    uint32_t rmask = 0;
#pragma unroll
    for (int blk = 0; blk < NBLK; ++blk)
#pragma unroll
        for (int k = 0; k < C; ++k)
            rmask |= (c0 + C * (8 * blk + l8) + k <= A.n1 ? 1u : 0u) << (C * blk + k);
    const int64_t rowb = timing ? 0 : A.pitch;  // int32 elements per table row
    int32_t *base = timing ? A.scratch + (int64_t)blockIdx.x * kScratchWords + 4 * g
                           : B.table + (c0 - A.tr_y0 + C * l8) * A.pitch + 4 * g;
    // GAP * (x + y) of element (blk, e, k) = kb + ug * (8 C blk + e + k) + ug * f
    const uint32_t kb = ug * (uint32_t)(4 * g) + ug * (uint32_t)(c0 + C * l8);
    const uint32_t bpos = (uint32_t)l8 * (4u * C);  // byte of compute lane a = 8 blk + l8 within its slot: + 32 C blk
    int32_t avail = 0;
    for (int32_t f = f0; f < nx; f += NS * BATCH) {
        const int32_t want = min(f + BATCH, nx);
        if (avail < want) {
            int32_t sa = __builtin_amdgcn_readfirstlane(ctr_load(ctr));
            if (sa != kDone && sa - 63 < want) sa = wait_counter(ctr, want + 63, A.ctrl, 8, A.timeout_ticks);
            avail = (sa == kDone || sa == kDead) ? nx : min(sa - 63, nx);
            lds_order();  // ring reads after the counter that released them
        }
        if (A.flags & NW_FLAG_DEBUG_DRAIN) {  // debug: drain the ring without reading it (compute-pace probe)
            lds_order();
            ctr_store(mine, f + NS * BATCH);
            continue;
        }
        VT v[NBLK][4];
#pragma unroll
        for (int blk = 0; blk < NBLK; ++blk)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t slot = (uint32_t)(f + 4 * g + e + 8 * blk + l8) & (uint32_t)(kR - 1);
                v[blk][e] = *(const VT *)(ring + slot * L::kSlot + bpos + (32u * C) * blk);
            }
        // the batch is in registers: release its ring rows before the stores
        lds_order();
        ctr_store(mine, f + NS * BATCH);
        if (plane) {  // the band's last row, columns f + 4g .. +3 (w form, as the ring holds it)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                uint32_t w = 0;
#pragma unroll
                for (int blk = 0; blk < NBLK; ++blk)
#pragma unroll
                    for (int k = 0; k < C; ++k)
                        if (blk == (pas >> 3) && k == pks) w = (uint32_t)comp<C>(v[blk][e], k);
                const int32_t x = f + 4 * g + e;
                if (x < nx) gran_store(A.feed_out + x, ptag | w);
            }
        }
        const bool xok = f + 4 * g <= A.n2;  // (a piece reaching past column n2 stays in the pitch slack)
        const uint32_t kf = kb + ug * (uint32_t)f;
        int32_t *col = timing ? base : base + f;
#pragma unroll
        for (int blk = 0; blk < NBLK; ++blk)
#pragma unroll
            for (int k = 0; k < C; ++k) {
                u32x4 o;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    o[e] = (uint32_t)comp<C>(v[blk][e], k) + kf + ug * (uint32_t)(8 * C * blk + e + k);
                if (xok && ((rmask >> (C * blk + k)) & 1u))
                    *(u32x4 *)(col + (int64_t)(8 * C * blk + k) * rowb) = o;
            }
    }
    ctr_store(mine, kDone);
}

// Store wave q of compute wave j on strip p, GROUPED ring (C == 1: 64 columns,
// records of 4 steps, lane slots gpos -- see grp_pos).  One store instruction
// covers 8 rows x 32 columns: lane (r, q8) = (lane / 8, lane % 8) takes row
// f + r, columns 32h + 4*q8 .. +3 (h = 0, 1: two instructions per 8 rows),
// gathered with 4 conflict-free ds_read_b32 (the value of column a of row f + r
// was computed at step f + r + a: record group (f+r+a)/4, word (f+r+a)%4).
// Rows go in batches of kBatch dealt round robin to the kSPR store waves.
template <int NC, bool TRACE>
__device__ __forceinline__ void store_strip_grp(const FillArgs &A, char *__restrict__ lds, const Blk &B,
                                                int j, int q, int lane) {
    const int p = B.pk;
    typedef Lay<1, NC> L;
    constexpr int BATCH = L::kBatch;  // a multiple of 8
    constexpr int NS = L::kSPR;
    constexpr int NU = BATCH / 8;     // 8-row units per batch
    constexpr uint32_t kMask = (uint32_t)L::kRing - 1u;
    int32_t *ctr = (int32_t *)(lds + L::kCtl) + j * L::kCtlWords;
    const uint32_t ring0 = (uint32_t)(j * L::kRing);
    const int64_t c0 = A.col0 + (int64_t)p * (NC * 64) + (int64_t)j * 64;
    const int32_t nrows = (int32_t)(A.n2 + 1);
    const bool timing = (A.flags & 1) != 0;
    const int ro = lane >> 3, cq = lane & 7;
    const int64_t rowb = timing ? 0 : A.pitch * 4;
    char *scr = (char *)(A.scratch + (int64_t)blockIdx.x * kScratchWords);
    const int32_t f0 = q * BATCH;
    const uint32_t ug = (uint32_t)A.gap;  // (both modes: the w form)
    // ring byte offset (within the ring) of column a = 32h + 4cq + k of row f0 + ro,
    // and kc = GAP * (row + column) of it (the ring holds w = t - GAP*(i+j))
    // The right half (columns 32..63) of a row completes 32 steps after the left
    // half, so a batch pairs the left halves of rows f .. f+BATCH-1 with the right
    // halves of rows f-32 .. f-32+BATCH-1: both are complete from step
    // f + BATCH - 1 + 32 on, and a ring slot (step x: column a of row x - a) is
    // free once the left halves of rows <= x and the right halves of rows <= x - 32
    // are read -- 32 steps earlier than with whole rows.
    constexpr int32_t kLagH = 32;
    uint32_t pa[2][4], kc[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t a = (uint32_t)(32 * h + 4 * cq + k);
            const uint32_t st = (uint32_t)(f0 + ro) + a + (h ? (uint32_t)(kR - kLagH) : 0u);  // (mod kR)
            pa[h][k] = (((st >> 2) * 1024u) & kMask) + grp_pos(a) * 16u + (st & 3u) * 4u;
            kc[h][k] = ug * (uint32_t)(f0 + ro - kLagH * h) + ug * (uint32_t)(c0 + a);
        }
    // the last strip may overhang the pitch: store only 16-byte pieces wholly inside the row
    bool col_ok[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) col_ok[h] = c0 + 32 * h + 4 * cq + 4 <= A.col_end;
    // SW: running maximum of this lane's cells (columns <= n1) for A.smax[p]
    uint32_t cval = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int k = 0; k < 4; ++k) cval |= (c0 + 32 * h + 4 * cq + k <= A.n1 ? 1u : 0u) << (4 * h + k);
    int32_t vmax = 0;
    char *rowp = timing ? scr : (char *)(B.table + c0) + (int64_t)f0 * rowb;
    const uint32_t voff = (uint32_t)(ro * rowb) + (uint32_t)cq * 16u;
    const bool bcol = A.col0 != 0 && p == 0 && j == 0 && !timing;
    int32_t bnd0 = 0;
    const int32_t *bnd0p = (const int32_t *)(lds + L::kCtl) + L::kStripWord + 1;
    int32_t *mine = ctr + 3 + q;
    if (A.flags & NW_FLAG_DEBUG_NO_STORE) {  // debug: no store waves at all (compute-pace probe, timing only)
        ctr_store(mine, kDone);
        return;
    }
    // debug trace (store wave 0 of ring 0): cycles waiting for rows / issuing stores
    const bool trace = TRACE && A.trace != nullptr && j == 0 && q == 0;
    uint64_t tw = 0, ts = 0;
    int32_t avail = 0;
    // batch f complete in the ring: left halves of rows < min(f + BATCH, nrows)
    // (step + 32) and right halves of rows < min(f - 32 + BATCH, nrows) (step + 64);
    // `avail` = steps known written (bounded wait)
    auto wait_rows = [&](int32_t f) {
        const int32_t want = max(min(f + BATCH, nrows) + 31, min(f - kLagH + BATCH, nrows) + 63);
        if (avail < want) {
            const uint64_t t0 = trace ? __builtin_amdgcn_s_memtime() : 0;
            int32_t sa = __builtin_amdgcn_readfirstlane(ctr_load(ctr));
            if (sa != kDone && sa < want) sa = wait_counter(ctr, want, A.ctrl, 8, A.timeout_ticks);
            avail = (sa == kDone || sa == kDead) ? INT32_MAX : sa;
            lds_order();
            if (bcol) bnd0 = *bnd0p;
            if (trace) tw += __builtin_amdgcn_s_memtime() - t0;
        }
    };
    // the next batch from the ring into v, raw (only the LDS reads are issued
    // here: nothing waits for them until the batch's own stores, one pipeline
    // stage later, so the stores of the previous batch go out while they are in
    // flight)
    auto read_batch = [&](u32x4 (&v)[NU][2]) {
#pragma unroll
        for (int g = 0; g < NU; ++g)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    v[g][h][k] = *(const uint32_t *)(lds + ring0 + ((pa[h][k] + g * 2048u) & kMask));
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int k = 0; k < 4; ++k) pa[h][k] = (pa[h][k] + (uint32_t)(NS * BATCH / 4) * 1024u) & kMask;
    };
    // stores of batch f (v from read_batch).  First the ring slots of every
    // batch read so far are released: `fr`, the last batch read (f, or f + D when
    // the next batch is already in registers); in-order LDS makes this counter
    // store execute after those reads.
    auto store_batch = [&](int32_t f, u32x4 (&v)[NU][2], int32_t fr) {
        lds_order();
        ctr_store(mine, fr + NS * BATCH);
        // t = w + GAP*(i+j): kc holds it for row f0 + ro; batch f adds GAP*(f - f0 + 8g)
        const uint32_t kf = ug * (uint32_t)(f - f0);
#pragma unroll
        for (int g = 0; g < NU; ++g)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int k = 0; k < 4; ++k) v[g][h][k] += kc[h][k] + kf + ug * (uint32_t)(8 * g);
        // row of unit g of half h: f + 8g + ro - 32h
        if (A.sw) {
            if (f >= kLagH && f + BATCH <= nrows && cval == 0xFFu) {  // interior batch
#pragma unroll
                for (int g = 0; g < NU; ++g)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int k = 0; k < 4; ++k) vmax = max(vmax, (int32_t)v[g][h][k]);
            } else {
#pragma unroll
                for (int g = 0; g < NU; ++g)
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int32_t r = f + g * 8 + ro - kLagH * h;
                        const bool rok = r >= 0 && r < nrows;
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            vmax = max(vmax, (rok && ((cval >> (4 * h + k)) & 1u)) ? (int32_t)v[g][h][k] : 0);
                    }
            }
        }
        const uint64_t t0 = trace ? __builtin_amdgcn_s_memtime() : 0;
        char *rp = rowp + (int64_t)(f - f0) * rowb;
        if (f >= kLagH && f + BATCH <= nrows) {
#pragma unroll
            for (int g = 0; g < NU; ++g)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (col_ok[h])
                        *(u32x4 *)(rp + (int64_t)(g * 8 - kLagH * h) * rowb + voff + h * 128) = v[g][h];
        } else {
#pragma unroll
            for (int g = 0; g < NU; ++g)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int32_t r = f + g * 8 + ro - kLagH * h;
                    if (col_ok[h] && r >= 0 && r < nrows)
                        *(u32x4 *)(rp + (int64_t)(g * 8 - kLagH * h) * rowb + voff + h * 128) = v[g][h];
                }
        }
        if (bcol) {
#pragma unroll
            for (int g = 0; g < NU; ++g) {
                const int32_t r = f + g * 8 + ro;
                if (cq == 0 && r < nrows)
                    *(int32_t *)(rp + (int64_t)g * 8 * rowb + (int64_t)voff - 4) = bnd0 + r * (A.sw ? 0 : (int32_t)ug);
            }
        }
        if (trace) ts += __builtin_amdgcn_s_memtime() - t0;
    };
    constexpr int32_t D = NS * BATCH;
    // Deadlock freedom of the pipeline: a store wave waits for batch f + D, i.e.
    // for step f + D + BATCH - 1 + 32, having released the slots of the steps
    // below f + D (at the stores of batch f - D, after reading batch f); the
    // compute wave writes that step once slots <= step + kChk - kR are free.
    static_assert(BATCH - 1 + 32 + L::kChk - kR <= 0, "store pipeline lookahead exceeds the ring");
    // batches run to f < nrows + 32: the right halves of the last 32 rows
    const int32_t fend = nrows + kLagH;
    if (A.flags & NW_FLAG_DEBUG_DRAIN) {  // debug: drain the ring without reading it
        for (int32_t f = f0; f < fend; f += D) {
            wait_rows(f);
            lds_order();
            ctr_store(mine, f + D);
        }
    } else if (f0 < fend) {
        // software pipeline over two register sets: batch f + D is read while
        // batch f is stored
        u32x4 va[NU][2], vb[NU][2];
        wait_rows(f0);
        read_batch(va);
        for (int32_t f = f0;; f += 2 * D) {
            if (f + D >= fend) {
                store_batch(f, va, f);
                break;
            }
            wait_rows(f + D);
            read_batch(vb);
            store_batch(f, va, f + D);
            if (f + 2 * D >= fend) {
                store_batch(f + D, vb, f + D);
                break;
            }
            wait_rows(f + 2 * D);
            read_batch(va);
            store_batch(f + D, vb, f + 2 * D);
        }
    }
    ctr_store(mine, kDone);
    if (A.sw) strip_max(A, p, vmax);
    if (trace && lane == 0) {
        uint64_t *trw = A.trace + (int64_t)(B.pq - A.strip0) * kTraceWords;
        trw[16] = tw;
        trw[17] = 0;
        trw[18] = ts;
    }
    // Row band: hand this ring's 64 columns of the last row to the next band (see
    // store_strip) -- from the store wave that stored the row's right half, the
    // later one; with kSPR = 1 for C = 1 that wave also stored the left half
    static_assert(NS == 1, "one store wave per grouped ring");
    if (B.halo_out != nullptr && ((nrows - 1 + kLagH) / BATCH) % NS == q && ctrl_load(A.ctrl + 1) == 0u) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const int32_t *last = B.table + A.n2 * A.pitch;
        const int64_t c = c0 + lane;
        if (c <= A.n1) {
            const uint32_t x = (uint32_t)__hip_atomic_load(last + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(B.halo_out + c, ((uint64_t)A.halo_tag << 32) | x, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (bcol && lane == 0)
            __hip_atomic_store(B.halo_out,
                               ((uint64_t)A.halo_tag << 32) | (uint32_t)(bnd0 + (int32_t)A.n2 * A.gap),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Strip shapes built with the Smith-Waterman modes (the tuned ones; the others
// refuse SW launches in nw_capi.cpp) -- each mode is a full copy of the loop.
constexpr bool sw_shape(int c, int nc) {
    return (c == 2 && nc == 2) || (c == 1 && nc == 4) || (c == 4 && nc == 1) || (c == 2 && nc == 1) ||
           (c == 2 && nc == 4);
}

// Kernel kinds: which two copies of the compute loop a kernel holds (the table form
// and a compare form; the choice between them is made on the device, from nprof).
// One kernel per kind rather than one holding every mode: each further copy of the
// unrolled loop, and the debug trace's stamps, raise the SGPR pressure of the whole
// kernel, which spills at the iteration boundaries (round 6: the generic (2, 2)
// kernel 485 spilled SGPRs with four modes and the trace, 136 for one kind without).
enum StripKind { KIND_GEN = 0, KIND_UNIT = 1, KIND_SW = 2 };

// Persistent grid of workgroups of NC compute waves (0 .. NC-1) and NC*kSPR
// store waves (wave NC + b serves ring b % NC).
template <int C, int NC, int KIND, bool TRACE>
__global__ __launch_bounds__((64 * Lay<C, NC>::kWaves)) void nw_fill_strips(FillArgs A) {
    typedef Lay<C, NC> L;
    static_assert(KIND != KIND_SW || sw_shape(C, NC), "Smith-Waterman kernel of a non-SW shape");
    static_assert(!L::kHalf || KIND == KIND_SW, "half-word rings hold Smith-Waterman cells only");
    __shared__ __attribute__((aligned(16))) char lds[L::kBytes];
    int32_t *ctl = (int32_t *)(lds + L::kCtl);
    const int lane = threadIdx.x & 63;
    // wave-uniform in an SGPR: every role / feed / output decision below is a
    // scalar branch (a divergent one would run the untaken side's spin-waits
    // with EXEC = 0, where they never see their counter)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (;;) {
        if (threadIdx.x == 0) {
            for (int w = 0; w < L::kStripWord; ++w) ctl[w] = 0;
            ctl[L::kFeedWord] = 0;
            ctl[L::kStripWord] = (int32_t)atomicAdd(A.ctrl, 1u);
        }
        __syncthreads();
        const int t = __builtin_amdgcn_readfirstlane(ctl[L::kStripWord]);
        if (t >= A.nstrips * A.nbl) break;
        const Blk B = make_blk(A, t);
        if (wave < NC) {
            // table form when the launch allows it (scores fit int8) and s1 has
            // at most kMaxPerm distinct characters (nw_charmap), else compares
            const uint32_t np = __builtin_amdgcn_readfirstlane(ctrl_load(A.nprof));
            const bool perm = A.perm != 0 && np <= kMaxPerm;
            if constexpr (KIND == KIND_SW) {
                if (perm)
                    compute_strip<C, NC, SUB_PERM_SW, TRACE>(A, lds, B, wave, lane);
                else
                    compute_strip<C, NC, SUB_GEN_SW, TRACE>(A, lds, B, wave, lane);
            } else if (perm) {
                compute_strip<C, NC, SUB_PERM, TRACE>(A, lds, B, wave, lane);
            } else if constexpr (KIND == KIND_UNIT) {
                compute_strip<C, NC, SUB_UNIT, TRACE>(A, lds, B, wave, lane);
            } else {
                compute_strip<C, NC, SUB_GEN, TRACE>(A, lds, B, wave, lane);
            }
        } else if (L::kFeeder && wave == L::kWaves - 1) {
            feed_strip<C, NC, TRACE>(A, lds, B, lane);
        } else {
            const int b = wave - NC;
            if constexpr (L::kGrp) {
                store_strip_grp<NC, TRACE>(A, lds, B, b % NC, b / NC, lane);
            } else if constexpr (((C == 4 && NC == 1) || (C == 2 && NC == 2)) && KIND != KIND_SW) {
                if (A.tr != 0)
                    store_strip_tr<C, NC>(A, lds, B, b % NC, b / NC, lane);  // (row band in horizontal strips)
                else
                    store_strip<C, NC>(A, lds, B, b % NC, b / NC, lane);
            } else {
                store_strip<C, NC>(A, lds, B, b % NC, b / NC, lane);
            }
        }
        __syncthreads();  // the rings and counters are reused by the next strip
    }
}
// The kernel of a launch: Smith-Waterman, or NW with match - mismatch = 1 (the
// compare form is then one add-with-carry), or NW generic; the trace build (only of
// the generic and SW kinds: a unit scheme's trace runs the generic kernel, whose
// table form is the same code) when FillArgs::trace is set.
template <int C, int NC>
static void launch_c(const FillArgs &a, int grid, hipStream_t s) {
    const dim3 block(64 * Lay<C, NC>::kWaves);
    const bool tr = a.trace != nullptr;
    if constexpr (sw_shape(C, NC)) {
        if (a.sw) {
            if (tr)
                hipLaunchKernelGGL((nw_fill_strips<C, NC, KIND_SW, true>), dim3(grid), block, 0, s, a);
            else
                hipLaunchKernelGGL((nw_fill_strips<C, NC, KIND_SW, false>), dim3(grid), block, 0, s, a);
            return;
        }
    }
    if constexpr (!Lay<C, NC>::kHalf) {  // (the host refuses NW on half-word rings)
        if (a.sw) return;                // (and SW on the shapes without an SW kernel)
        if (tr)
            hipLaunchKernelGGL((nw_fill_strips<C, NC, KIND_GEN, true>), dim3(grid), block, 0, s, a);
        else if (a.match - a.mismatch == 1)
            hipLaunchKernelGGL((nw_fill_strips<C, NC, KIND_UNIT, false>), dim3(grid), block, 0, s, a);
        else
            hipLaunchKernelGGL((nw_fill_strips<C, NC, KIND_GEN, false>), dim3(grid), block, 0, s, a);
    }
}

}  // namespace nw
