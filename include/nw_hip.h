/*
 * nw_hip.h -- C ABI of libnwhip.so, the MI355X (gfx950) Needleman-Wunsch fill.
 *
 * This is the drop-in boundary for the reference's fill plugins.  The reference
 * selects a fill at link time: every fill TU defines
 *
 *     void needlemanWunsch(dnaArray s1, dnaArray s2, int* t);
 *       src/serial/serial.cpp:4          (serial -- the oracle)
 *       src/sentinel/sentinel-mt.cpp:4   (sentinel-mt)
 *       src/idxarray/idxarray-mt.cpp:4   (idxarray-mt)
 *
 * and textually includes src/common/driver.cpp (its main(), :1-40).  The
 * MI355X drop-in TU (fast-needleman-wunsch_amd/dropin/needleman-wunsch-hip.cpp)
 * defines that same C++ symbol and forwards to nw_fill() below.  Everything in
 * this header is plain C: pointers, sizes, PODs -- no HIP or torch types.
 *
 * Table layout (reference contract, serial.cpp:6-7,21-31): nRows = n2 + 1
 * (s2 "down the side"), nCols = n1 + 1 (s1 "across the top"), cell (i, j) at
 * t[i * nCols + j], int32.  On the device the library may use a row pitch
 * >= nCols (see nw_table_pitch); host copies always use the reference layout.
 */
#ifndef NW_HIP_H
#define NW_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (the reference's fill is void and cannot fail; the C ABI reports
 * what the device path can: bad arguments, HIP errors, OOM, a watchdog trip) */
enum {
    NW_OK = 0,
    NW_ERR_ARG = 1,       /* invalid argument (sizes, pitch, alignment, mode)   */
    NW_ERR_HIP = 2,       /* a HIP runtime call failed                         */
    NW_ERR_OOM = 3,       /* device allocation failed / table does not fit     */
    NW_ERR_TIMEOUT = 4,   /* a bounded in-kernel wait expired (never expected) */
    NW_ERR_NODEVICE = 5,  /* no gfx950 device visible                          */
    NW_ERR_UNSUPPORTED = 6
};

/* nw_params.mode: global alignment (the reference fills) or Smith-Waterman local
 * alignment (BASELINE config 5; no reference counterpart -- conventions in
 * nw_sw_align below) */
enum { NW_MODE_NW = 0, NW_MODE_SW = 1 };

/* nw_params.flags (0 = normal fill) */
enum {
    NW_FLAG_TIMING_ONLY = 1, /* table stores go to a scratch tile (kernel timing only) */
    NW_FLAG_NO_PROFILE = 2,  /* substitution by byte compares instead of the per-lane
                                v_perm score tables */
    NW_FLAG_NO_FINISH = 4,   /* nw_fill_tband_async: sweep every row in strips, also a
                                last strip that runs alone as one more pass (default:
                                such rows go to the row-scan finisher) */
    /* debug probes of the compute pace: only together with NW_FLAG_TIMING_ONLY
       (refused otherwise -- the table is not written) */
    NW_FLAG_DEBUG_DRAIN = 0x100,    /* store waves drain the LDS ring without reading it */
    NW_FLAG_DEBUG_NO_STORE = 0x200, /* no store waves at all */
    /* store-pattern probe (strip kernel, no halo / feed): every strip takes the
       boundary column instead of its left neighbour's and publishes nothing, so the
       strips run unchained; the table IS written to HBM but holds no fill (refused
       on bands and in NW_MODE_SW, whose best cell would be meaningless) */
    NW_FLAG_DEBUG_NO_CHAIN = 0x400,
    /* with NO_CHAIN: strip p of a one-pass launch starts p * 11.5 us after it is
       claimed -- the chained sweep's diagonal, without its hand-offs */
    NW_FLAG_DEBUG_STAGGER = 0x800
};

/* nw_params.kernel: which gfx950 kernel family fills the table.  Both compute
 * the same cells (serial.cpp:21-33); they differ in how the wavefront maps onto
 * a wave:
 *   STRIPS: a wave holds an ANTI-DIAGONAL of a 64*C-column strip (lane = row
 *           offset; DPP carries the left neighbour), rows leave through a
 *           128-slot LDS ring.  Shapes (substrips C, strip_waves NC): (4,1)
 *           (2,1) (1,1) (2,2) (1,2) (1,4); and (2,4), Smith-Waterman only: 512-
 *           column strips on half-word rings, refused (NW_ERR_UNSUPPORTED) when
 *           more than 64 cells could reach 2^16 (max(match, mismatch) * min(i, j)
 *           >= 65536), which are then recomputed exactly after the fill.
 *   PANELS: a wave holds a ROW of 64*C columns, computed as a prefix maximum
 *           (lane-local prefix + a 64-lane DPP max-scan) in the w form; rows
 *           leave through a 32-row ring.  Shapes (C, NW compute waves per
 *           panel): (4,4) (4,2) (2,4) (4,1) (2,2) (1,4).
 *   AUTO:   with substrips = strip_waves = 0, the measured family and shape
 *           for the table size (nw_auto_shape); with an explicit shape, STRIPS.
 *           Smith-Waterman, row-band and column-band AUTO fills use the strips. */
enum { NW_KERNEL_AUTO = 0, NW_KERNEL_STRIPS = 1, NW_KERNEL_PANELS = 2 };

/* Runtime replacement for the compile-time constants of
 * src/common/needleman-wunsch.hpp:11-13 (MATCH 1, MISMATCH 0, GAP -1). */
typedef struct nw_params {
    int32_t match;     /* default  1 */
    int32_t mismatch;  /* default  0 */
    int32_t gap;       /* default -1 */
    int32_t mode;      /* NW_MODE_NW */
    int32_t waves;     /* persistent strip workers (waves; 0 = auto)     */
    int32_t device;    /* HIP device ordinal, -1 = current device         */
    int32_t flags;     /* NW_FLAG_* bits, 0 for a normal fill            */
    int32_t substrips; /* columns per lane C of a compute wave (1, 2 or 4); 0 = auto */
    int32_t strip_waves; /* chained compute waves per strip NC (1, 2 or 4); 0 = auto.
                            A strip is NC * 64 * C columns; supported (C, NC):
                            (4,1) (2,1) (1,1) (2,2) (1,2) (1,4), SW also (2,4)
                            (see NW_KERNEL_AUTO); auto = the tuned
                            shape for the size (nw_tuned_shape) */
    int32_t timeout_ms;  /* bound of every in-kernel wait (hand-off, halo, ring);
                            0 = 20000.  A wait that expires makes the fill return
                            NW_ERR_TIMEOUT instead of hanging the device. */
    int32_t kernel;      /* NW_KERNEL_*; 0 = auto.  With PANELS, substrips /
                            strip_waves are the panel's (C, NW): a panel is
                            NW * 64 * C columns */
} nw_params;

typedef struct nw_result {
    int32_t score;          /* t[n2][n1] -- what driver.cpp:35 prints     */
    int32_t status;         /* NW_OK or an error code                     */
    int64_t cells;          /* n1 * n2 inner cells (GCUPS numerator)      */
    double kernel_ms;       /* device time of the fill (HIP events)       */
    double table_bytes;     /* bytes of table stored: 4 * nRows * nCols   */
    int32_t strips;         /* strips swept (64 * substrips * strip_waves columns each) */
    int32_t waves;          /* persistent workers launched                */
    int32_t substrips;      /* columns per lane of a compute wave         */
    int32_t strip_waves;    /* compute waves per strip                    */
    int64_t end_i, end_j;   /* cell `score` was read from: (n2, n1) for NW; for SW
                               the best cell, first in row-major order     */
    int32_t kernel;         /* NW_KERNEL_STRIPS or NW_KERNEL_PANELS (what ran) */
    int32_t reserved;
} nw_result;

/* A Smith-Waterman alignment (nw_sw_align / nw_sw_traceback). */
typedef struct nw_alignment {
    int32_t score;           /* t[end_i][end_j], the table maximum            */
    int32_t status;
    int64_t begin_i, begin_j; /* cell where the traceback reached t == 0      */
    int64_t end_i, end_j;    /* best cell (first row-major maximum)          */
    int64_t n_ops;           /* ops written, path order begin -> end          */
    double fill_ms, traceback_ms;
} nw_alignment;

/* Fill `p` with the reference defaults (1, 0, -1). */
void nw_params_default(nw_params *p);

/* Human-readable text for a status code. */
const char *nw_strerror(int status);

/* Library / kernel build identification (gfx target, kernel variant). */
const char *nw_version(void);

/*
 * One-shot fill from host buffers (the drop-in path).  Copies s1/s2 to the
 * device, fills the whole table in HBM, and -- when host_t != NULL -- copies
 * the table back in the reference layout (nCols-pitched, (n2+1)*(n1+1) ints).
 * With host_t == NULL only the score is returned.  Returns NW_OK or an error.
 * Replaces needlemanWunsch() of serial.cpp:4 / sentinel-mt.cpp:4 /
 * idxarray-mt.cpp:4 (called from driver.cpp:28).
 */
int nw_fill(const int8_t *s1, int64_t n1, const int8_t *s2, int64_t n2,
            const nw_params *p, int32_t *host_t, nw_result *out);

/*
 * nw_fill, nw_fill_emb and nw_sw_align keep per-device state between calls: a
 * context, the device table (kept when at most 16 GiB) and sequence buffers,
 * and three pinned staging chunks (up to 256 MiB each) through which the
 * table is copied back (DMA of the next chunks overlapping the threaded copy of
 * one into host_t; NW_COPY_THREADS sets the copy threads, default min(8, cores)).
 * nw_host_warmup(device) creates it ahead of the first call (context, copy
 * stream, staging; not the table, whose size is not known yet; -1: the current
 * device); nw_host_release(device) frees it (-1: every device).
 * NW_HOST_TIMING=1 prints nw_fill's phases (prepare, fill, copy back) to stderr.
 */
int nw_host_warmup(int device);
void nw_host_release(int device);

/*
 * The same fill into the "emb" table layout of the reference's second driver
 * (src/common/driver2.cpp:20-22 allocates (s1.size+2) * (s2.size+1) ints;
 * src/idxarray/idxarray-emb-mt.cpp:4-65 fills it): rows of n1+2 ints, column 0
 * = each row's progress counter at its final value n1+2, columns 1 .. n1+1 = the
 * serial table.  host_t is required.
 */
int nw_fill_emb(const int8_t *s1, int64_t n1, const int8_t *s2, int64_t n2,
                const nw_params *p, int32_t *host_t, nw_result *out);

/*
 * Smith-Waterman local alignment with on-device traceback (BASELINE config 5).
 * Table: t[i][0] = t[0][j] = 0, t[i][j] = max(0, t[i-1][j-1] + s, t[i-1][j] + GAP,
 * t[i][j-1] + GAP) (gap <= 0).  Best cell: the maximum, first in row-major
 * order.  Traceback from it while t > 0, preferring diag > up > left (the order
 * of serial.cpp:24-30's max).  ops[k] (path order, begin -> end): 0 = diagonal
 * (s1[j-1] against s2[i-1]), 1 = up (s2[i-1] against a gap), 2 = left (s1[j-1]
 * against a gap); ops_cap >= n1 + n2 always suffices.  p->mode must be
 * NW_MODE_SW.  The reference has no local alignment: parity is against the
 * build's CPU restatement (oracle/nw_oracle.c), not the reference.
 */
int nw_sw_align(const int8_t *s1, int64_t n1, const int8_t *s2, int64_t n2, const nw_params *p,
                uint8_t *ops, int64_t ops_cap, nw_alignment *out);

/* Device-resident API ------------------------------------------------------ */
typedef struct nw_ctx nw_ctx;

/* Strip shape (columns per lane C, chained compute waves NC) that a fill with
 * nw_params.substrips = strip_waves = 0 uses for an n1 x n2 table: the table
 * measured by tools/tune.py (the analogue of the reference's block tuner,
 * src/common/block-tuner.cpp:26-34, src/block-tune.sh). */
void nw_tuned_shape(int64_t n1, int64_t n2, int32_t *substrips, int32_t *strip_waves);

/* Kernel family and shape a global-alignment fill with kernel = substrips =
 * strip_waves = 0 uses for an n1 x n2 table on a device with `cus` compute units
 * (hipDeviceProp_t.multiProcessorCount): the same measured table, whose panel
 * entries apply only when every CU gets a panel (n1 + 1 >= cus * 64 * C * NW). */
void nw_auto_shape(int64_t n1, int64_t n2, int32_t cus, int32_t *kernel, int32_t *substrips,
                   int32_t *strip_waves);

/* Row pitch (in int32 elements) the library allocates for nCols = n1+1: a
 * multiple of 64 (256-byte rows) with at least 3 columns of slack after column
 * n1, which the strips need to start at column 1 (nw_table_offset).  Any
 * multiple of 64 >= n1 + 1 is accepted; a tighter one sweeps from column 0. */
int64_t nw_table_pitch(int64_t n1);

/* Bytes of device memory a table of (n2+1) rows at nw_table_pitch(n1) takes. */
int64_t nw_table_bytes(int64_t n1, int64_t n2);

/* Preferred element offset of the table base from a 256-byte aligned
 * allocation (of nw_table_bytes + 256 bytes): 63, which puts column 1 of every
 * row on a 256-byte line.  The fill then sweeps columns 1..n1 only -- an
 * N x N table is exactly N / 256 strips -- and stores the boundary column 0
 * separately.  A 256-byte aligned base (offset 0) is accepted too. */
int64_t nw_table_offset(void);

/* LDS bytes of one strip workgroup of shape (C = substrips, NC = strip_waves),
 * -1 for an unsupported shape.  A CU holds floor(160 KiB / this) of them; a
 * caller co-scheduling several fills on one device (LocalBands) sizes their
 * `waves` from it so that all of them stay resident. */
int64_t nw_strip_lds_bytes(int32_t substrips, int32_t strip_waves);
/* LDS bytes of one PANEL workgroup (NW_KERNEL_PANELS) of shape (C, NW); -1 if
 * unsupported. */
int64_t nw_panel_lds_bytes(int32_t substrips, int32_t strip_waves);

/* Create / destroy a context bound to `device` (-1 = current).  The context
 * owns the hand-off workspace and the strip ticket counter. */
int nw_ctx_create(int device, nw_ctx **out);
void nw_ctx_destroy(nw_ctx *ctx);

/* Workspace bytes the context will allocate for this shape (advisory). */
int64_t nw_ctx_workspace_bytes(int64_t n1, int64_t n2, int32_t waves);

/*
 * Fill a device-resident table.  d_s1/d_s2: device int8 sequences; d_t: device
 * table with row pitch `pitch` (a multiple of 64 >= n1 + 1; nw_table_pitch
 * preferred), base 256-byte aligned or -- preferred -- 4 bytes short of it
 * (nw_table_offset; used when pitch >= n1 + 4).
 * `stream` is a hipStream_t (NULL = default stream).
 * Asynchronous with respect to the host unless out != NULL, in which case the
 * call synchronises the stream and fills `out` (score read back from HBM).
 */
int nw_fill_device(nw_ctx *ctx, const int8_t *d_s1, int64_t n1,
                   const int8_t *d_s2, int64_t n2, const nw_params *p,
                   int32_t *d_t, int64_t pitch, void *stream, nw_result *out);

/* Traceback of a device-resident SW table filled by nw_fill_device /
 * nw_fill_device_async (mode SW) from (end_i, end_j) (nw_result.end_i/end_j);
 * ops copied to the host as in nw_sw_align.  Synchronous: it first waits for
 * all work on the device (the fill may be on any stream).  `p` must be a valid
 * SW parameter set (mode NW_MODE_SW), else NW_ERR_ARG. */
int nw_sw_traceback(nw_ctx *ctx, const int8_t *d_s1, int64_t n1, const int8_t *d_s2, int64_t n2,
                    const nw_params *p, const int32_t *d_t, int64_t pitch, int64_t end_i, int64_t end_j,
                    uint8_t *ops, int64_t ops_cap, nw_alignment *out);

/* Launch-only variant for timing loops: no synchronisation, no readback. */
int nw_fill_device_async(nw_ctx *ctx, const int8_t *d_s1, int64_t n1,
                         const int8_t *d_s2, int64_t n2, const nw_params *p,
                         int32_t *d_t, int64_t pitch, void *stream);

/* Row bands (multi-GPU) ---------------------------------------------------
 * The reference's 8-GPU twin is src/mpi/mpi-horz.cpp:4-99 (+ mpi-horz-driver.cpp):
 * rank r fills a contiguous band of rows whose row 0 is rank r-1's last row (the
 * halo), received in chunks while r-1 is still filling.  Here band r's kernel
 * takes that row from `halo_in` -- granules {tag:32 | value:32}, one per column
 * 0..n1 -- as each strip (64 * substrips * strip_waves columns) starts, and
 * publishes its own last row into
 * `halo_out` (the next band's halo_in, usually peer memory on the next GPU
 * mapped with nw_ipc_open_handle) as each strip finishes: a pipelined halo with
 * no host round trip.  `tag` identifies the launch (> 0, the same value on both
 * sides of a halo, new for every launch); halo buffers must start zeroed. */
typedef struct nw_band {
    const uint64_t *halo_in;  /* NULL: row 0 is the boundary j*gap (first band)  */
    uint64_t *halo_out;       /* NULL: last band                                  */
    uint32_t tag;
    uint32_t row0;            /* global row index of the band's row 0 (nw_band_layout
                                 `start`): bounds the cell values for the range check */
} nw_band;

/* Band layout of mpi-horz-driver.cpp:31-32: rows of band r (including its halo
 * row) and the global index of its row 0, for a table of n2+1 rows in nbands. */
void nw_band_layout(int64_t n2, int32_t nbands, int32_t r, int64_t *n_rows, int64_t *start);

/* Bytes of one halo granule buffer for n1 (+1) columns. */
int64_t nw_halo_bytes(int64_t n1);

/* A zeroed halo granule buffer of its own hipMalloc (so that nw_ipc_get_handle
 * exports exactly it); device -1 = current. */
int nw_halo_alloc(int device, int64_t n1, uint64_t **d_halo);
int nw_halo_free(uint64_t *d_halo);

/* Fill one band: d_t holds n2_band+1 rows (row 0 = the halo row, written by
 * the kernel from halo_in), d_s2_band = the band's side characters
 * (s2 + start of the band: local row i >= 1 uses d_s2_band[i-1]).  Async. */
int nw_fill_band_async(nw_ctx *ctx, const int8_t *d_s1, int64_t n1, const int8_t *d_s2_band,
                       int64_t n2_band, const nw_params *p, const nw_band *band, int32_t *d_t,
                       int64_t pitch, void *stream);

/* Block-cyclic row bands (the config-4 row-band case, pipelined) --------------
 * Same contract as nw_fill_band_async (mpi-horz.cpp:4-99: a block's row 0 is the
 * previous block's last row, streamed strip by strip), but the table's rows are
 * cut into P * nblk blocks of n2_blk rows dealt round robin to the P ranks --
 * global block g = k * P + r is rank r's block k -- so that every rank is busy
 * after P blocks instead of waiting for P - 1 whole bands.  One launch fills all
 * of a rank's blocks, strips claimed in (block, strip) order:
 *   * block k's table is d_t + k * t_stride (each laid out like a band: n2_blk + 1
 *     rows, row 0 = the halo row), its side characters d_s2_blocks + k * n2_blk;
 *   * its halo row comes from region k of halo_in (regions of nw_halo_bytes(n1),
 *     nw_halo_alloc_regions) -- block 0 only if hin_first (rank 0: block 0's
 *     row 0 is the boundary);
 *   * its last row goes to region k + hout_shift of halo_out (the next rank's
 *     halo_in; hout_shift = 1 on the last rank, whose block k feeds rank 0's
 *     block k + 1; regions >= nblk are not written).  With P = 1, halo_out =
 *     halo_in and hout_shift = 1 chain a rank's blocks through its own buffer.
 * Strip kernel only (NW_ERR_UNSUPPORTED for panels). */
typedef struct nw_band_cycle {
    const uint64_t *halo_in;
    uint64_t *halo_out;
    int32_t nblk;
    int32_t hin_first;
    int32_t hout_shift;
    uint32_t tag;             /* as nw_band.tag                                       */
    int64_t row0_max;         /* global row of the last block's row 0 (range check)   */
    int64_t t_stride;         /* int32 elements between blocks' tables (>= (n2_blk+1) * pitch,
                                 a multiple of 64)                                     */
} nw_band_cycle;

int nw_halo_alloc_regions(int device, int64_t n1, int32_t nregions, uint64_t **d_halo);
int nw_fill_band_cycle_async(nw_ctx *ctx, const int8_t *d_s1, int64_t n1, const int8_t *d_s2_blocks,
                             int64_t n2_blk, const nw_params *p, const nw_band_cycle *cy, int32_t *d_t,
                             int64_t pitch, void *stream);

/* Column bands (multi-GPU, n1 >> n2) ------------------------------------------
 * The reference's twin is src/mpi/mpi-vert.cpp:4-109 (+ mpi-vert-driver.cpp:35-38):
 * rank r fills a contiguous band of columns whose column 0 is rank r-1's last
 * column, received in COMMBUF_SIZE-row chunks while r-1 is still filling.  Here
 * the bands are whole strips of the global table's sweep (strips of
 * W = 64 * substrips * strip_waves columns starting at column 1): band r owns
 * strips [strip_first, strip_first + strip_count) and its local table holds
 * global columns [start, start + n_cols), start = strip_first * W, so local
 * column 0 is band r-1's last column as in mpi-vert.  The first strip of band
 * r > 0 takes that column from `feed_in` as band r-1's last strip produces it
 * (granules {tag:32 | value:32}, one per row, nw_feed_bytes), and band r's last
 * strip publishes its right column into `feed_out` (band r+1's feed_in, usually
 * peer memory mapped with nw_ipc_open_handle) row block by row block.  After
 * the fill, local column 0 of band r > 0 is written from feed_in.  Every band
 * must use the same n1, n2 and strip shape (explicit substrips / strip_waves, or
 * 0/0 = the tuned shape of the whole n1 x n2 table); NW mode only. */
typedef struct nw_colband {
    const uint64_t *feed_in;  /* NULL: first band (column 0 = the boundary i*gap) */
    uint64_t *feed_out;       /* NULL: last band                                  */
    uint32_t tag;             /* launch tag (> 0, the same on both sides of a feed,
                                 new for every launch; not the value of any other
                                 launch's tag on these buffers)                    */
    int32_t nbands;           /* bands of the table                               */
    int32_t r;                /* this band                                        */
    int32_t reserved;
} nw_colband;

/* Layout of band r of nbands over an n1 x n2 table with the strip shape of `p`:
 * its strips and the global column range of its local table (local column 0 =
 * global column start).  Returns NW_ERR_ARG when nbands exceeds the strips. */
int nw_colband_layout(int64_t n1, int64_t n2, int32_t nbands, int32_t r, const nw_params *p,
                      int64_t *strip_first, int64_t *strip_count, int64_t *start, int64_t *n_cols);

/* Bytes of one feed granule buffer for n2 (+1) rows, and a zeroed one of its own
 * hipMalloc (exportable by nw_ipc_get_handle); free with nw_halo_free. */
int64_t nw_feed_bytes(int64_t n2);
int nw_feed_alloc(int device, int64_t n2, uint64_t **d_feed);

/* Fill column band band->r: d_s1 / d_s2 the WHOLE sequences (n1 / n2); d_t the
 * band's local table laid out like nw_table_offset's (n_cols - 1 = its "n1"),
 * pitch >= nw_table_pitch(n_cols - 1).  Asynchronous on `stream`. */
int nw_fill_colband_async(nw_ctx *ctx, const int8_t *d_s1, int64_t n1, const int8_t *d_s2,
                          int64_t n2, const nw_params *p, const nw_colband *band, int32_t *d_t,
                          int64_t pitch, void *stream);

/* Row bands in HORIZONTAL strips (the config-4 row-band case, short chain) ----
 * The same contract and partition as nw_fill_band_async (src/mpi/mpi-horz.cpp:4-99,
 * nw_band_layout: band r's row 0 is band r-1's last row) and the same row-major
 * band table, but the band is swept the other way round: its rows are cut into
 * strips of 256 rows that run left to right along the columns, one step per
 * column (the (4, 1) strip kernel on the transposed band, whose store waves
 * write the row-major table in 128-byte row pieces).  Band r's first strip takes
 * row 0 from `feed_in` column by column as band r-1's last strip produces it
 * (granules {tag:32 | w:32}, one per column 0..n1: nw_feed_alloc(device, n1)), and
 * band r's last strip publishes its last row into `feed_out`.  Band r+1 therefore
 * starts 256 rows (a strip's 64-column hop) after band r instead of after band
 * r's whole height -- the reference streams its halo in 1280-column chunks for
 * the same reason (mpi-horz.cpp:28-40).  After the fill, row 0 is written from
 * feed_in (the boundary j*gap for band 0) and column 0 is the boundary i*gap.
 * d_t: (n2_band + 1) rows laid out like nw_table_offset's (column 1 starts a
 * 256-byte line), pitch >= nw_table_pitch(n1); d_s2_band: the band's n2_band side
 * characters (global rows row0 + 1 ..).  NW mode, strip shapes (4, 1) (the default,
 * nw_params.substrips = strip_waves = 0) and (2, 2) -- 256 rows either way
 * (NW_ERR_UNSUPPORTED otherwise).  Asynchronous on `stream`. */
/* nw_tband.flags */
enum {
    /* the band's waiting strips poll their feed with s_sleep 1 instead of s_sleep 64
       between polls (and the chain's leader is not throttled): a shorter strip-to-strip
       lag (10.0 vs 12.2-12.5 us) at a slower leading strip (28.0-28.5 vs 26.8-27.2 ms) --
       the better choice for chains of more than ~520 strips (2+ bands of 65536 rows;
       DESIGN.md section 5) */
    NW_TBAND_DENSE_POLLS = 1
};
typedef struct nw_tband {
    const uint64_t *feed_in;  /* NULL: first band (row 0 = the boundary j*gap)     */
    uint64_t *feed_out;       /* NULL: last band                                    */
    uint32_t tag;             /* launch tag, as nw_colband.tag                      */
    uint32_t flags;           /* NW_TBAND_* (0: sparse polls); unknown bits refused */
    int64_t row0;             /* global row of the band's row 0 (nw_band_layout start;
                                 0 exactly when feed_in is NULL)                    */
} nw_tband;

int nw_fill_tband_async(nw_ctx *ctx, const int8_t *d_s1, int64_t n1, const int8_t *d_s2_band,
                        int64_t n2_band, const nw_params *p, const nw_tband *band, int32_t *d_t,
                        int64_t pitch, void *stream);

/* Cross-process device pointers (one process per GPU): export a device
 * allocation, open a peer's export.  Handles are NW_IPC_HANDLE_BYTES bytes. */
#define NW_IPC_HANDLE_BYTES 64
int nw_ipc_get_handle(const void *d_ptr, void *handle);
int nw_ipc_open_handle(const void *handle, void **d_ptr);
int nw_ipc_close_handle(void *d_ptr);

/* Launch-to-launch flow control between neighbouring bands -------------------
 * A band sweep that enqueues K fills back to back (no host round trip between
 * them) alternates two halo / feed buffers by launch parity, so the producer's
 * launch k + 2 must not start before the consumer's launch k has read buffer
 * k % 2.  The consumer signals "done with launch k" into a LINK word that lives
 * in the producer's memory (a peer store over xGMI), the producer's stream waits
 * on it.  (The reference's blocking MPI_Send / MPI_Recv pairs,
 * src/mpi/mpi-horz.cpp:41-42,53-54, give the same ordering per chunk.)
 * nw_link_alloc: a zeroed 256-byte fine-grained word pair of its own allocation
 *   (exportable by nw_ipc_get_handle; free with nw_halo_free).
 * nw_link_wait_async: stream-ordered wait until word[0] >= value (wrapping
 *   compare); after timeout_ms (0 = 20000) it gives up and records value in
 *   word[1].
 * nw_link_wait_ctx_async: the same, and a wait that gives up also records the
 *   failure in ctx (code 4): ctx's next fill then gives up at once, without
 *   publishing into the buffer its consumer has not released, and nw_ctx_status
 *   reports NW_ERR_TIMEOUT.
 * nw_link_signal_async: stream-ordered word[0] = value (word may be peer memory).
 * nw_link_status: word[1] (0 = no wait gave up), read synchronously. */
int nw_link_alloc(int device, uint32_t **d_word);
int nw_link_wait_async(uint32_t *d_word, uint32_t value, int32_t timeout_ms, void *stream);
int nw_link_wait_ctx_async(nw_ctx *ctx, uint32_t *d_word, uint32_t value, int32_t timeout_ms, void *stream);
int nw_link_signal_async(uint32_t *d_word, uint32_t value, void *stream);
int nw_link_status(const uint32_t *d_word, uint32_t *out);

/* NW_ERR_TIMEOUT if ANY launch on ctx since the previous call gave up (an
 * in-kernel watchdog, or a nw_link_wait_ctx_async that expired), else NW_OK;
 * syncs the stream and clears the record.  Until it is read, a recorded failure
 * makes every later launch on ctx give up at once (a back-to-back sweep stops
 * at its first failure instead of waiting out one watchdog per launch). */
int nw_ctx_status(nw_ctx *ctx, void *stream);

/* Debug hooks (diagnosis, not needed for fills).
 * nw_debug_ctrl: the 8 control words of the context's last launch: [0] strip
 *   ticket, [1] error code (0 ok; 1 hand-off granule wait -- strips, panels, the
 *   finisher's look-back (site 30) --, 2 halo wait, 3 LDS counter wait expired), [2] site << 24 | wave << 16 | address bits, [3] the
 *   value the wait needed, [4] the value it last saw.  Syncs the device.  (A
 *   launch that a recorded failure made give up carries that failure's words.)
 * nw_debug_failure: the first failure recorded on ctx -- code (1 granule wait,
 *   2 halo wait, 3 LDS counter, 4 link wait), site word, need, seen, and the
 *   number of failed launches (the failing one and every launch it poisoned) -- pending, or as the last nw_ctx_status cleared it.
 * nw_debug_set_trace: per-strip timeline buffer (device memory of at least
 *   strips * nw_debug_trace_words() uint64), NULL = off. */
int nw_debug_ctrl(nw_ctx *ctx, uint32_t *out8);
int nw_debug_failure(nw_ctx *ctx, uint32_t *out5);
int nw_debug_set_trace(nw_ctx *ctx, void *d_trace);
int32_t nw_debug_trace_words(void);

/* Host helpers ------------------------------------------------------------- */

/* readSequence semantics (src/common/helper.cpp:3-25): every byte of the file,
 * no stripping.  *out is malloc'ed; free with nw_free().  Returns NW_OK or
 * NW_ERR_ARG if the file cannot be opened. */
int nw_read_bdna(const char *path, int8_t **out, int64_t *n);
void nw_free(void *p);

/* Seeded synthetic sequence: i.i.d. uniform bytes in {1,2,3,4} (SplitMix64). */
void nw_synth_bdna(uint64_t seed, int64_t n, int8_t *out);

#ifdef __cplusplus
}
#endif
#endif /* NW_HIP_H */
