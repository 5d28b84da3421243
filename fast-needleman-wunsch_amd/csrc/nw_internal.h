// nw_internal.h -- shared between the HIP kernels (nw_fill.hip) and the C-ABI
// layer (nw_capi.cpp).  Not part of the public ABI (include/nw_hip.h is).
#pragma once
#include <stdint.h>

#include "nw_hip.h"  // (nw_params flag bits the kernels test)

namespace nw {

constexpr int kWave = 64;          // lanes per wavefront
constexpr int kQOff = 64;          // rowpack index offset (lane l reads index 4g - l)
constexpr int32_t kNeg = -(1 << 29);  // "minus infinity" fed left of column 0
constexpr int kScratchWords = kWave * kWave + 2 * kWave;  // per workgroup (16.5 KB)
constexpr int kMaxSub = 4;        // max columns per lane (strip = 64 * C columns)
constexpr int kTraceWords = 24;    // debug trace words per strip (nw_debug_trace_words)
constexpr uint32_t kMaxPerm = 7;  // distinct column characters the v_perm score tables cover
constexpr int kMetaBytes = 256 + 16 + 32;  // charmap[256], nprof (+ pad), present[8] (zero between launches)

// Everything one launch of the strip-sweep kernel needs.  Plain POD, passed by
// value as the kernel argument.
struct FillArgs {
    int32_t *table;            // device table, row-major, row pitch `pitch` (int32 elems)
    int64_t pitch;             // multiple of 64 (256-B aligned rows)
    const void *rowpack;       // 16-byte entries: rowpack[x + kQOff] = B[x .. x+15],
                               //   B[x] = s2[x-1] for 1 <= x <= n2, else 0 (raw or
                               //   mapped through charmap: nw_rowpack)
    const uint8_t *s1;         // n1 column characters
    int64_t n1, n2;            // nCols = n1 + 1, nRows = n2 + 1
    int64_t row0;              // global row index of local row 0 (0 for a whole table)
    int64_t col0;              // first swept column: 1 when column 1 starts a 256-B line
                               //   (column 0 = the boundary, stored separately), else 0
    int32_t nstrips;           // strips: ceil((nCols - col0) / (strip_waves * 64 * substrips))
    int32_t nblocks;           // ceil(nRows / 64)
    uint64_t *gran;            // right-boundary hand-off granules [M][gstride] {tag:32 | value:32}
    int64_t gstride;           // granules per slot = 64 * nblocks
    int32_t M;                 // number of slots (>= waves + 1, or nstrips)
    uint32_t tagbase;          // strip p publishes tag tagbase + p + 1
    uint32_t *ctrl;            // [0] strip ticket, [1] error word, [2..4] watchdog site/need/seen
    // Row bands (mpi-horz contract): row 0 of this launch is the previous band's
    // last row, delivered as granules {tag:32 | value:32}, one per column 0..n1.
    const uint64_t *halo_in;   // NULL = row 0 is the boundary j*gap (first band / whole table)
    uint64_t *halo_out;        // NULL, or the next band's halo_in (peer memory): row n2 goes here
    uint32_t halo_tag;         // launch tag shared with the neighbouring bands (> 0)
    int32_t *scratch;          // per-workgroup dummy flush target: grid * kScratchWords int32
    uint64_t *trace;           // optional per-strip debug trace [nstrips][kTraceWords]
    // v_perm score tables (SUB_PERM): allowed by the host when s - GAP fits
    // int8 for both scores; used when s1 has <= kMaxPerm distinct characters.
    // charmap / nprof are written on the device by launch_rowpack (nw_charmap).
    int32_t perm;
    const uint8_t *charmap;
    const uint32_t *nprof;
    int32_t match, mismatch, gap;
    int32_t flags;             // debug: bit0 = send table stores to the scratch tile (timing only)
    uint64_t timeout_ticks;    // bound of every in-kernel wait (s_memrealtime ticks, 100 MHz)
    // Smith-Waterman (local alignment): cells t = max(0, ...), row/column 0 = 0;
    // store waves fold each strip's best cell into smax[p] (zeroed before launch)
    int32_t sw;
    int32_t *smax;
    // Column bands (mpi-vert contract): this launch sweeps global strips
    // strip0 .. strip0 + nstrips - 1 of the table; `table` is biased so that
    // table + c addresses global column c, and stores stay below column col_end.
    // feed_in: the left neighbour band's last strip's right column (granules
    // {tag:32 | w:32}, gstride of them, NULL = strip0's feed is the internal one
    // or the boundary); feed_out: where this launch's last strip publishes its
    // right column (peer memory; NULL = internal slot).  Both carry feed_tag.
    int32_t strip0;
    int64_t col_end;
    const uint64_t *feed_in;
    uint64_t *feed_out;
    uint32_t feed_tag;
    // Block-cyclic row bands (nw_fill_band_cycle_async): the launch sweeps nbl
    // row blocks of n2 + 1 rows one after the other (strips claimed in (block,
    // strip) order); block b's table is table + b * tstride, its row packs
    // rowpack + b * qstride bytes, its halo row region b of halo_in (block 0 only
    // if hin0) and its last row goes to region b + hoshift of halo_out (if that
    // is < nbl).  Strip slots and tags run over the whole launch.  nbl = 1,
    // hin0 = 1, hoshift = 0: one table (every other launch).
    int32_t nbl;
    int32_t hin0, hoshift;
    int64_t tstride, qstride, hstride;
    // Row band in HORIZONTAL strips (nw_fill_tband_async): the launch sweeps the
    // transposed band -- its strips run along the band's rows, one step per
    // table column -- so `n1` / `s1` / col0 above describe the band's ROWS in
    // global row numbers (col0 = first swept global row, s1 biased so that
    // s1[y - 1] is global row y's character) and `n2` / the row packs its
    // columns.  Store waves write the real row-major band table (`table`, row 0 =
    // global row tr_y0).  The feeds carry the band's top row in and its last row
    // out; tr_pub is the strip-local column of that last row in the last strip.
    int32_t tr;
    int32_t tr_pub;
    int32_t tr_store_pub;  // 1: the last strip's store waves publish the band's last row
                           // (0: its compute wave, NW_TR_PUB_COMPUTE=1 for A/B)
    int64_t tr_y0;
    // the unfed leading strip sleeps lead_sleep x 64 clocks per 64-step iteration
    // (horizontal (4, 1) strips: 8, nw_capi.cpp kTbandLeadSleep; NW_LEAD_SLEEP overrides)
    int32_t lead_sleep;
    // horizontal strips: 1 = waiting strips poll with s_sleep 1 (NW_TBAND_DENSE_POLLS)
    int32_t tr_dense;
};
bool sw_shape_ok(int substrips, int strip_waves);
// column band r > 0: local column 0 (global column `start`) from the feed
// granules, t = w + gap * (i + start), rows 0..n2; asynchronous on `stream`
int launch_colband_edge(const uint64_t *feed, int32_t *table, int64_t pitch, int64_t n2, int32_t gap,
                        int64_t start, void *stream);
// horizontal-strip row band: row 0 (x = 0..n1; from the feed granules, w form,
// or the boundary x*gap when feed is NULL) and column 0 (rows 1..rows-1:
// (start + y)*gap) of the band table; asynchronous on `stream`
int launch_tband_edges(const uint64_t *feed, int32_t *table, int64_t pitch, int64_t n1, int64_t rows,
                       int32_t gap, int64_t start, void *stream);
// best cell of an SW table: reduce smax[nstrips] and find the first row-major cell
// holding the maximum (out8[0] = score, out8[1..2] = row, out8[3..4] = column as
// 64-bit halves); device buffers, asynchronous on `stream`
int launch_sw_locate(const int32_t *table, int64_t pitch, int64_t n1, int64_t n2, int64_t col0,
                     int32_t strip_cols, const int32_t *smax, int32_t nstrips, uint64_t *key, int32_t *best,
                     void *stream);
// half-word strip rings (Lay::kHalf, Smith-Waterman): the corner i, j >= k whose
// cells may reach 2^16 (*k = ceil(2^16 / max(match, mismatch))) and its cell count
int64_t sw_half_corner(int32_t match, int32_t mismatch, int64_t n1, int64_t n2, int64_t *k);
// cells the host lets the half-word shape leave to nw_sw_fixup (above: refused)
constexpr int64_t kHalfFixMax = 64;
// recompute that corner exactly after a half-word fill and raise the strips'
// best-cell words to its values (asynchronous on `stream`, before launch_sw_locate)
int launch_sw_fixup(int32_t *table, int64_t pitch, int64_t n1, int64_t n2, const uint8_t *s1, const uint8_t *s2,
                    int32_t match, int32_t mismatch, int32_t gap, int64_t col0, int32_t strip_cols, int32_t *smax,
                    void *stream);
// traceback from (end_i, end_j), parallel over row windows (nw_sw.hip): ops[]
// gets one byte per move from the end cell back (0 diag, 1 up, 2 left); host
// info[0] = moves, [1..2] = begin cell, [3] = status (0 ok, 1 ops buffer too
// small, 2 not a Smith-Waterman table), [4] rounds, [5] windows.  Synchronises
// `stream` once per round.  scratch: sw_tb_scratch_bytes(maxwin, band) bytes.
size_t sw_tb_scratch_bytes(int32_t maxwin, int32_t band);
int run_sw_traceback(const int32_t *table, int64_t pitch, int64_t n1, const uint8_t *s1, const uint8_t *s2,
                     int32_t match, int32_t mismatch, int32_t gap, int64_t end_i, int64_t end_j, uint8_t *ops,
                     int64_t ops_cap, void *scratch, int32_t maxwin, int32_t band, int64_t *info, void *stream);
constexpr int32_t kTbBandDefault = 256;    // band half-width of the traceback windows (profiles/r03s_tb_geometry.txt)
constexpr int32_t kTbMaxWinDefault = 512;  // windows per round (64 rows each)

// Launch helpers implemented in nw_fill.hip.  Return hipError_t as int.
// charmap of s1 into meta, then the row packs (mapped when perm allows it)
int launch_rowpack(const uint8_t *d_s1, int64_t n1, const uint8_t *d_s2, int64_t n2, int64_t row0,
                   int32_t perm, uint8_t *meta, void *d_q, int64_t qlen, void *stream);
bool shape_ok(int substrips, int strip_waves);
int launch_fill(const FillArgs &a, int substrips, int strip_waves, int grid, void *stream);
int lds_bytes(int substrips, int strip_waves);
// Row-scan panels (nw_rows.hip): shapes (C columns per lane, NW compute waves)
bool panel_shape_ok(int c, int nwaves);
int panel_lds_bytes(int c, int nwaves);
int launch_panels(const FillArgs &a, int c, int nwaves, int grid, void *stream);
// Band-to-band flow control (nw_link.hip): wait until word[0] >= value (word[1]
// records a timeout), or store word[0] = value; one-lane kernels on `stream`
int launch_link_wait(uint32_t *word, uint32_t value, uint64_t ticks, uint32_t *poison, void *stream);
// reset a context's per-launch control words, keeping (and re-raising) its
// recorded failure (nw_link.hip nw_ctrl_reset)
int launch_ctrl_reset(uint32_t *ctrl, void *stream);
constexpr int kCtrlWords = 16;
int launch_link_signal(uint32_t *word, uint32_t value, void *stream);

// Row-scan finisher (nw_finish.hip): rows li0 .. li0 + nrows - 1 of a row band
// (local row 0 = global row grow0), every column 1..n1, each row a prefix
// maximum in the w form with a decoupled look-back over column chunks.
struct FinishArgs {
    int32_t *table;            // band table, row-major (column 1 on a 256-byte line)
    int64_t pitch;
    const uint8_t *s1;         // column characters (n1)
    int64_t n1;
    const uint8_t *s2;         // the band's side characters: local row li uses s2[li - 1]
    int64_t li0, nrows, grow0;
    int32_t match, mismatch, gap;
    uint64_t *look;            // [nrows][nchunks] look-back granules {tag, value}
    uint32_t tag0;             // row r: aggregate tag0 + 2r, inclusive tag0 + 2r + 1 (unique per launch)
    int32_t nchunks, chunk_cols;
    uint32_t *ctrl;            // the context's control words: [1] error word, [6] chunk ticket
    uint64_t *feed_out;        // the next band's feed (w form, one granule per column), or NULL
    uint32_t feed_tag;
    uint64_t timeout_ticks;
};
int finish_chunk_cols(int64_t n1, int cus);  // columns per chunk (256 threads x 8 or x 32)
int launch_finish_rows(const FinishArgs &a, void *stream);
int64_t rowpack_len(int32_t nblocks);  // 16-byte entries
const char *kernel_variant();

}  // namespace nw
