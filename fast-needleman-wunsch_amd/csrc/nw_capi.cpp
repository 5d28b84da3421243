// nw_capi.cpp -- C ABI of libnwhip.so (declared in include/nw_hip.h).
//
// Owns device workspace (hand-off granules, row-character packs, ticket/error
// words, ramp scratch), validates shapes, and launches the gfx950 kernels of
// nw_fill.hip.  The one-shot nw_fill() is the drop-in path used by the
// reference-signature TU (dropin/needleman-wunsch-hip.cpp); it replaces the
// reference fills' needlemanWunsch() (serial.cpp:4, sentinel-mt.cpp:4,
// idxarray-mt.cpp:4) as called from driver.cpp:28.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "nw_hip.h"
#include "nw_internal.h"
#include "nw_tuned.h"

struct nw_ctx {
    int device = 0;
    int cus = 256;
    uint64_t *gran = nullptr;
    size_t gran_cap = 0;  // bytes
    void *rowpack = nullptr;
    size_t rowpack_cap = 0;
    uint8_t *meta = nullptr;   // charmap / nprof (nw::kMetaBytes)
    int32_t *scratch = nullptr;
    size_t scratch_cap = 0;
    uint32_t *ctrl = nullptr;  // nw::kCtrlWords: [0..7] per launch, [8..12] failure since the last status read
    uint32_t tagbase = 1;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int last_waves = 0;
    int last_strips = 0;
    int last_sub = 0;
    int last_nc = 0;
    uint64_t *trace = nullptr;  // debug: per-strip timestamps (nw_debug_set_trace)
    int32_t *smax = nullptr;    // SW: per-strip best cell + best / key words
    size_t smax_cap = 0;
    uint8_t *ops = nullptr;     // SW traceback ops (device)
    size_t ops_cap = 0;
    int64_t *swinfo = nullptr;  // SW locate key ([12])
    void *tbscratch = nullptr;  // SW traceback windows (nw::sw_tb_scratch_bytes)
    size_t tbscratch_cap = 0;
    int last_col0 = 0;
    int last_kernel = NW_KERNEL_STRIPS;
    uint32_t last_failure[5] = {0, 0, 0, 0, 0};  // ctrl[8..12] as the last nw_ctx_status read them
    uint64_t *look = nullptr;   // row-scan finisher look-back granules (nw_finish.hip)
    size_t look_cap = 0;
    uint32_t look_tag = 1;
    int last_finish_rows = 0;   // rows the last horizontal-band launch left to the finisher
};

namespace {

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

#define NW_HIP_TRY(expr)                                                         \
    do {                                                                         \
        hipError_t e_ = (expr);                                                  \
        if (e_ != hipSuccess) {                                                  \
            std::fprintf(stderr, "libnwhip: %s failed: %s (%s:%d)\n", #expr,     \
                         hipGetErrorString(e_), __FILE__, __LINE__);             \
            return e_ == hipErrorOutOfMemory ? NW_ERR_OOM : NW_ERR_HIP;          \
        }                                                                        \
    } while (0)

// (Re)allocate a workspace buffer; returns NW_OK and sets *fresh when it is new.
int grow(void **p, size_t *cap, size_t need, bool *fresh = nullptr) {
    if (fresh) *fresh = false;
    if (need <= *cap) return NW_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    need = (size_t)round_up((int64_t)need, 1 << 21);
    NW_HIP_TRY(hipMalloc(p, need));
    *cap = need;
    if (fresh) *fresh = true;
    return NW_OK;
}

struct Shape {
    int64_t nRows, nCols, nstrips, nblocks, waves, M, gstride;
    int64_t waves_max;  // resident strip workgroups (before capping at nstrips)
    int32_t K, NC;
    int32_t kernel;     // NW_KERNEL_STRIPS or NW_KERNEL_PANELS
};

constexpr int kLdsPerCU = 160 * 1024;

// Strip shape for nw_params.substrips = strip_waves = 0: the measured table of
// tools/tune.py (csrc/nw_tuned.h, by table size), else (2, 2).  The table is
// measured on squares.  A table at least 4x wider than tall is bound by the
// chain of strip-to-strip hand-offs (strips x hop latency) rather than by its
// stores, and wants the shape with the shortest hop: measured with
// tools/rect_time.py, 524288 x 8191 fills in 15.5 ms with (4,1) against 19.9
// (2,2) and 29.7 (1,4); 524288 x 65535 in 33.0 ms with (2,2), 33.7 (4,1), 37.4 (1,4).
void tuned_shape(int64_t n1, int64_t n2, int32_t *c, int32_t *nc, int32_t *kernel = nullptr, int cus = 0) {
    const double cells = (double)(n1 + 1) * (double)(n2 + 1);
    *c = 2;
    *nc = 2;
    if (kernel) *kernel = NW_KERNEL_STRIPS;
    if (n1 + 1 >= 4 * (n2 + 1) && n1 >= 65536) {
        *c = n2 + 1 <= 32768 ? 4 : 2;
        *nc = n2 + 1 <= 32768 ? 1 : 2;
        return;
    }
    // a panel entry applies only when every CU gets a panel in one pass (the
    // table is measured on squares; a tall narrow table with as many cells would
    // leave CUs idle) -- otherwise the last strip entry that applies stands
    for (const auto &e : nw::kTuned) {
        if (cells < e.min_cells) continue;
        if (e.kernel == NW_KERNEL_PANELS) {
            if (!kernel || !nw::panel_shape_ok(e.c, e.nc) || n1 + 1 < (int64_t)cus * nw::kWave * e.c * e.nc) continue;
            *kernel = NW_KERNEL_PANELS;
        } else {
            if (!nw::shape_ok(e.c, e.nc)) continue;
            if (kernel) *kernel = NW_KERNEL_STRIPS;
        }
        *c = e.c;
        *nc = e.nc;
    }
}

// col0: first swept column (1 when the table's column 1 starts a 256-byte line)
// Panel shape for nw_params.kernel = PANELS with substrips = strip_waves = 0:
// the widest panel that still gives every CU a panel (a panel is one CU's
// work; the 256k square has 262144 / 1024 = 256 of (4,4)).
void panel_auto(int64_t n1, int cus, int32_t *c, int32_t *nw) {
    const int64_t cols = n1 + 1;
    if (cols >= (int64_t)cus * 1024) {
        *c = 4;
        *nw = 4;
    } else if (cols >= (int64_t)cus * 512) {
        *c = 2;
        *nw = 4;
    } else {
        *c = 4;
        *nw = 1;
    }
}

Shape make_shape(int64_t n1, int64_t n2, int32_t waves_req, int32_t sub_req, int32_t nc_req,
                 int cus, int64_t col0, bool sw = false, int32_t kernel_req = NW_KERNEL_AUTO) {
    Shape s;
    s.kernel = kernel_req == NW_KERNEL_PANELS ? NW_KERNEL_PANELS : NW_KERNEL_STRIPS;
    if (kernel_req == NW_KERNEL_AUTO && sub_req <= 0 && nc_req <= 0 && !sw) {
        // the measured choice of kernel family and shape (csrc/nw_tuned.h)
        tuned_shape(n1, n2, &s.K, &s.NC, &s.kernel, cus);
    } else if (s.kernel == NW_KERNEL_PANELS) {
        if (sub_req <= 0 && nc_req <= 0) {
            panel_auto(n1, cus, &s.K, &s.NC);
        } else {
            s.K = sub_req > 0 ? sub_req : 4;
            s.NC = nc_req > 0 ? nc_req : 4;
        }
    } else if (sub_req <= 0 && nc_req <= 0 && sw) {
        // Smith-Waterman cells cost 4 VALU instead of 2, which moves the balance
        // toward more compute waves: 65536^2 (tools/sw_shapes.py) (2,2) 7.15 ms,
        // (4,1) 7.57, (2,1) 7.95, (1,4) 8.64
        s.K = 2;
        s.NC = 2;
    } else if (sub_req <= 0 && nc_req <= 0) {
        tuned_shape(n1, n2, &s.K, &s.NC);
    } else {
        s.K = sub_req > 0 ? sub_req : 2;
        s.NC = nc_req > 0 ? nc_req : (s.K == 1 ? 4 : s.K == 2 ? 2 : 1);
    }
    s.nRows = n2 + 1;
    s.nCols = n1 + 1;
    const int64_t width = (int64_t)nw::kWave * s.K * s.NC;
    s.nstrips = std::max<int64_t>(1, (s.nCols - col0 + width - 1) / width);
    s.nblocks = (s.nRows + nw::kWave - 1) / nw::kWave;
    // one strip workgroup per LDS ring set; as many as fit in a CU's LDS (a
    // panel workgroup is 2 * NW waves: at most 32 waves per CU)
    const int lds = s.kernel == NW_KERNEL_PANELS ? nw::panel_lds_bytes(s.K, s.NC) : nw::lds_bytes(s.K, s.NC);
    int64_t per_cu = std::max(1, kLdsPerCU / std::max(lds, 1));
    // a panel workgroup (NW compute, 2-3 store waves per compute wave, 2 feeder
    // waves, ~88 VGPRs each) fills a CU's wave slots on its own
    if (s.kernel == NW_KERNEL_PANELS) per_cu = 1;
    int64_t w = waves_req > 0 ? waves_req : per_cu * cus;
    s.waves_max = std::max<int64_t>(1, w);
    s.waves = std::max<int64_t>(1, std::min<int64_t>(w, s.nstrips));
    // Strip p publishes into slot p % M.  When strip p is claimed, every strip
    // <= p - waves has finished, so M = waves + 1 slots never alias a live one.
    s.M = std::min<int64_t>(s.nstrips, s.waves + 1);
    s.gstride = s.nblocks * nw::kWave;
    return s;
}

// Row / column band fills: AUTO means the strips (the tuned table is measured
// on whole square tables, and a band's geometry is set by its caller).
int32_t band_kernel(int32_t k) { return k == NW_KERNEL_AUTO ? NW_KERNEL_STRIPS : k; }

bool fits_i8(int32_t x) { return x >= -128 && x <= 127; }

bool shape_valid(const Shape &s) {
    return s.kernel == NW_KERNEL_PANELS ? nw::panel_shape_ok(s.K, s.NC) : nw::shape_ok(s.K, s.NC);
}

bool valid_params(const nw_params *p) {
    if (!p) return false;
    if (p->mode != NW_MODE_NW && p->mode != NW_MODE_SW) return false;
    if (p->mode == NW_MODE_SW && p->gap > 0) return false;  // local alignment needs a penalty
    if (p->substrips != 0 && p->substrips != 1 && p->substrips != 2 && p->substrips != 4) return false;
    if (p->strip_waves != 0 && p->strip_waves != 1 && p->strip_waves != 2 && p->strip_waves != 4 &&
        p->strip_waves != 8)
        return false;
    if (p->kernel != NW_KERNEL_AUTO && p->kernel != NW_KERNEL_STRIPS && p->kernel != NW_KERNEL_PANELS) return false;
    if (p->timeout_ms < 0) return false;
    // known flag bits only; the debug probes leave the table unwritten, so only with TIMING_ONLY
    const int32_t dbg = NW_FLAG_DEBUG_DRAIN | NW_FLAG_DEBUG_NO_STORE;
    if ((p->flags & ~(NW_FLAG_TIMING_ONLY | NW_FLAG_NO_PROFILE | NW_FLAG_NO_FINISH | NW_FLAG_DEBUG_NO_CHAIN |
                      NW_FLAG_DEBUG_STAGGER | dbg)) != 0)
        return false;
    if ((p->flags & NW_FLAG_DEBUG_STAGGER) && !(p->flags & NW_FLAG_DEBUG_NO_CHAIN)) return false;
    if ((p->flags & dbg) != 0 && (p->flags & NW_FLAG_TIMING_ONLY) == 0) return false;
    // keep every intermediate far from int32 overflow (|score| < 2^29)
    const int32_t lim = 1 << 12;
    return std::abs(p->match) < lim && std::abs(p->mismatch) < lim && std::abs(p->gap) < lim;
}

}  // namespace

extern "C" {

void nw_params_default(nw_params *p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->match = 1;      // needleman-wunsch.hpp:11
    p->mismatch = 0;   // needleman-wunsch.hpp:12
    p->gap = -1;       // needleman-wunsch.hpp:13
    p->mode = NW_MODE_NW;
    p->waves = 0;
    p->device = -1;
}

const char *nw_strerror(int status) {
    switch (status) {
        case NW_OK: return "ok";
        case NW_ERR_ARG: return "invalid argument";
        case NW_ERR_HIP: return "HIP runtime error";
        case NW_ERR_OOM: return "out of device memory";
        case NW_ERR_TIMEOUT: return "in-kernel hand-off watchdog expired";
        case NW_ERR_NODEVICE: return "no gfx950 device";
        case NW_ERR_UNSUPPORTED: return "unsupported";
        default: return "unknown status";
    }
}

const char *nw_version(void) {
    static char buf[256];
    std::snprintf(buf, sizeof buf, "libnwhip gfx950 %s", nw::kernel_variant());
    return buf;
}

// nCols = n1 + 1 rounded up to 64, with >= 3 columns of slack after column n1 so
// that the 16-byte store holding column n1 stays inside the row when the strips
// start at column 1 (nw_table_offset)
int64_t nw_table_pitch(int64_t n1) { return round_up(n1 + 4, nw::kWave); }

int64_t nw_table_bytes(int64_t n1, int64_t n2) {
    return round_up(n2 + 1, nw::kWave) * nw_table_pitch(n1) * (int64_t)sizeof(int32_t);
}

int64_t nw_table_offset(void) { return nw::kWave - 1; }

int64_t nw_strip_lds_bytes(int32_t substrips, int32_t strip_waves) {
    if (!nw::shape_ok(substrips, strip_waves)) return -1;
    return nw::lds_bytes(substrips, strip_waves);
}

int64_t nw_panel_lds_bytes(int32_t substrips, int32_t strip_waves) {
    if (!nw::panel_shape_ok(substrips, strip_waves)) return -1;
    return nw::panel_lds_bytes(substrips, strip_waves);
}

int64_t nw_ctx_workspace_bytes(int64_t n1, int64_t n2, int32_t waves) {
    Shape s = make_shape(n1, n2, waves, 0, 0, 256, 1);
    return s.M * s.gstride * 8 + nw::rowpack_len((int32_t)s.nblocks) * 16 +
           s.waves * nw::kScratchWords * 4 + 16;
}

int nw_ctx_create(int device, nw_ctx **out) {
    if (!out) return NW_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return NW_ERR_NODEVICE;
    if (device < 0) NW_HIP_TRY(hipGetDevice(&device));
    if (device >= ndev) return NW_ERR_ARG;
    NW_HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    NW_HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        std::fprintf(stderr, "libnwhip: device %d is %s, kernels are built for gfx950\n", device,
                     prop.gcnArchName);
        return NW_ERR_NODEVICE;
    }
    nw_ctx *c = new nw_ctx();
    c->device = device;
    c->cus = prop.multiProcessorCount;
    if (hipMalloc(&c->ctrl, nw::kCtrlWords * 4) != hipSuccess || hipMemset(c->ctrl, 0, nw::kCtrlWords * 4) != hipSuccess ||
        hipMalloc(&c->meta, nw::kMetaBytes) != hipSuccess || hipMemset(c->meta, 0, nw::kMetaBytes) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        nw_ctx_destroy(c);
        return NW_ERR_HIP;
    }
    *out = c;
    return NW_OK;
}

void nw_ctx_destroy(nw_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->gran) (void)hipFree(c->gran);
    if (c->rowpack) (void)hipFree(c->rowpack);
    if (c->meta) (void)hipFree(c->meta);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->ctrl) (void)hipFree(c->ctrl);
    if (c->smax) (void)hipFree(c->smax);
    if (c->ops) (void)hipFree(c->ops);
    if (c->swinfo) (void)hipFree(c->swinfo);
    if (c->tbscratch) (void)hipFree(c->tbscratch);
    if (c->look) (void)hipFree(c->look);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    delete c;
}

// Column band r of nbands (nw_colband_layout): strips [sf, sf + sc) of the whole
// table's sweep (col0 = 1), local column 0 = global column start = sf * W.
static int colband_layout(int64_t n1, int64_t n2, int32_t nb, int32_t r, const nw_params *p, int cus,
                   int64_t *sf, int64_t *sc, int64_t *start, int64_t *ncols) {
    if (!p || n1 < 1 || n2 < 0 || nb < 1 || r < 0 || r >= nb) return NW_ERR_ARG;
    const Shape s = make_shape(n1, n2, 0, p->substrips, p->strip_waves, cus, 1, false, band_kernel(p->kernel));
    if (!shape_valid(s) || nb > s.nstrips) return NW_ERR_ARG;
    const int64_t W = (int64_t)nw::kWave * s.K * s.NC;
    const int64_t base = s.nstrips / nb, extra = s.nstrips % nb;
    *sf = r * base + std::min<int64_t>(r, extra);
    *sc = base + (r < extra ? 1 : 0);
    *start = *sf * W;
    *ncols = std::min(*sc * W, n1 - *start) + 1;  // + the left column (band r-1's last)
    return NW_OK;
}

static int launch_fill(nw_ctx *c, const int8_t *d_s1, int64_t n1, const int8_t *d_s2, int64_t n2,
                       const nw_params *p, const nw_band *band, const nw_colband *cb, int32_t *d_t,
                       int64_t pitch, void *stream, const nw_band_cycle *cy = nullptr) {
    if (!c || !d_t || n1 < 0 || n2 < 0 || n1 >= INT32_MAX || n2 >= INT32_MAX) return NW_ERR_ARG;
    // block-cyclic row bands: nbl blocks of n2 + 1 rows, checked as a band whose
    // row 0 is the largest of the blocks'
    nw_band cyb;
    const int32_t nbl = cy ? cy->nblk : 1;
    if (cy) {
        if (band || cb || cy->nblk < 1 || (cy->hin_first & ~1) != 0 || (cy->hout_shift & ~1) != 0 ||
            cy->row0_max < 0 || cy->row0_max >= INT32_MAX)
            return NW_ERR_ARG;
        if (!cy->halo_in && (cy->hin_first || cy->nblk > 1)) return NW_ERR_ARG;
        if (cy->nblk > 1 && (cy->t_stride < (n2 + 1) * pitch || cy->t_stride % nw::kWave != 0)) return NW_ERR_ARG;
        if ((int64_t)nbl * n2 >= INT32_MAX) return NW_ERR_ARG;
        cyb.halo_in = cy->halo_in;
        cyb.halo_out = cy->halo_out;
        cyb.tag = cy->tag;
        cyb.row0 = (uint32_t)cy->row0_max;
        band = &cyb;
    }
    if ((n1 > 0 && !d_s1) || (n2 > 0 && !d_s2)) return NW_ERR_ARG;
    if (!valid_params(p)) return NW_ERR_ARG;
    const bool sw = p->mode == NW_MODE_SW;
    if (sw && (band || cb)) return NW_ERR_UNSUPPORTED;  // (local alignment: single table, config 5)
    // the unchained probe leaves no valid table, so no best cell / locate either
    if (sw && (p->flags & NW_FLAG_DEBUG_NO_CHAIN)) return NW_ERR_ARG;
    if ((p->flags & NW_FLAG_DEBUG_NO_CHAIN) && (band || cb)) return NW_ERR_ARG;  // (no fill to hand on)
    if (band && cb) return NW_ERR_ARG;
    // The kernels hold w = t - GAP*(i+j) in int32 next to a "minus infinity" of
    // -2^29: |w| <= (max|score| + |GAP|) * (i + j) must stay below 2^28, with i the
    // GLOBAL row (a band's halo row carries the values of row band->row0).  The same
    // bound holds for Smith-Waterman: its cells are in the w form too (strips: the
    // 0 floor becomes z = -GAP*(i+j); panels: u = t - GAP*j), so |w|, |z| and the
    // store waves' GAP*(i+j) reach (max|score| + |GAP|) * (n1 + n2 + 2) although t
    // itself stays in [0, max|score| * (min(n1, n2) + 1)].
    {
        const long long m = std::max({std::llabs(p->match), std::llabs(p->mismatch), std::llabs(p->gap)});
        const long long i_max = (long long)n2 + (band ? (long long)band->row0 : 0);
        if ((m + std::llabs(p->gap)) * (long long)(n1 + i_max + 2) >= (1LL << 28)) return NW_ERR_ARG;
    }
    int64_t col0;
    int64_t strip_first = 0, strip_count = 0, start = 0;
    if (cb) {
        // a column band's local table: the nw_table_offset layout over its n_cols
        // columns (local column 1 starts a 256-byte line, as in every band)
        if (cb->tag == 0 || (((uintptr_t)cb->feed_in | (uintptr_t)cb->feed_out) & 7u) != 0) return NW_ERR_ARG;
        int64_t ncols = 0;
        int st0 = colband_layout(n1, n2, cb->nbands, cb->r, p, c->cus, &strip_first, &strip_count, &start, &ncols);
        if (st0 != NW_OK) return st0;
        if ((cb->r > 0) != (cb->feed_in != nullptr) || (cb->r + 1 < cb->nbands) != (cb->feed_out != nullptr))
            return NW_ERR_ARG;
        if (cb->feed_out && (p->flags & 1)) return NW_ERR_ARG;  // needs the real right column
        if ((((uintptr_t)d_t + 4u) & 255u) != 0 || pitch % nw::kWave != 0 || pitch < ncols + 3) return NW_ERR_ARG;
        col0 = 1;
    } else {
        // any 64-multiple pitch that holds nCols = n1 + 1 (nw_table_pitch adds the
        // slack that lets the strips start at column 1)
        if (pitch < n1 + 1 || pitch % nw::kWave != 0) return NW_ERR_ARG;
        // Strip origin: column 1 when the base is laid out so that column 1 starts a
        // 256-byte line (nw_table_offset), which takes the boundary column 0 out of
        // the sweep; column 0 for a 256-byte aligned base.  Anything else is refused.
        if ((((uintptr_t)d_t + 4u) & 255u) == 0 && n1 >= 1 && pitch >= n1 + 4)
            col0 = 1;
        else if (((uintptr_t)d_t & 255u) == 0)
            col0 = 0;
        else
            return NW_ERR_ARG;
    }
    if (band) {
        if (band->tag == 0 || (((uintptr_t)band->halo_in | (uintptr_t)band->halo_out) & 7u) != 0)
            return NW_ERR_ARG;
        if (band->halo_out && (p->flags & 1)) return NW_ERR_ARG;  // needs the real last row
    }
    NW_HIP_TRY(hipSetDevice(c->device));
    Shape s = make_shape(n1, n2, p->waves, p->substrips, p->strip_waves, c->cus, col0, sw,
                         band || cb ? band_kernel(p->kernel) : p->kernel);
    if (!shape_valid(s)) return NW_ERR_ARG;
    const bool panels = s.kernel == NW_KERNEL_PANELS;
    if (cy && panels) return NW_ERR_UNSUPPORTED;  // (block cycles: the strip kernel)
    if (panels && (p->flags & NW_FLAG_DEBUG_NO_CHAIN)) return NW_ERR_ARG;  // (a strip-kernel probe)
    if ((int64_t)s.nstrips * nbl > INT32_MAX / 2) return NW_ERR_ARG;
    if (nbl > 1) {  // the launch's chain of hand-offs is nstrips * nbl tickets long
        s.waves = std::max<int64_t>(1, std::min<int64_t>(s.waves_max, s.nstrips * nbl));
        s.M = std::min<int64_t>(s.nstrips * nbl, s.waves + 1);
    }
    if (cb) {  // this launch sweeps its band's strips only
        s.nstrips = strip_count;
        s.waves = std::max<int64_t>(1, std::min<int64_t>(s.waves_max, s.nstrips));
        s.M = std::min<int64_t>(s.nstrips, s.waves + 1);
    }
    if (sw && !panels && !nw::sw_shape_ok(s.K, s.NC)) return NW_ERR_UNSUPPORTED;
    // (2, 4): half-word rings, Smith-Waterman only, with at most kHalfFixMax cells of
    // the corner where t may reach 2^16 (nw_sw.hip nw_sw_fixup)
    const bool half = !panels && s.K == 2 && s.NC == 4;
    if (half) {
        int64_t k = 0;
        if (!sw || nw::sw_half_corner(p->match, p->mismatch, n1, n2, &k) > nw::kHalfFixMax) return NW_ERR_UNSUPPORTED;
    }
    if (s.nstrips > INT32_MAX / 2 || s.nblocks > INT32_MAX / 2) return NW_ERR_ARG;

    int st;
    // Hand-off granules.  (Re)allocation zeroes them; tags are then unique per
    // (launch, strip) as long as tagbase does not wrap -- re-zero when it would.
    // A new buffer is zeroed on the launch stream (ordered before the kernels
    // below on any stream, also a non-blocking one): reused device memory may
    // still hold granules whose tags match this context's fresh tagbase.
    const size_t gran_need = (size_t)(s.M * s.gstride) * sizeof(uint64_t);
    bool fresh = false;
    if ((st = grow((void **)&c->gran, &c->gran_cap, gran_need, &fresh)) != NW_OK) return st;
    if (fresh) {
        NW_HIP_TRY(hipMemsetAsync(c->gran, 0, c->gran_cap, (hipStream_t)stream));
        c->tagbase = 1;
    }
    // tags run up to tagbase + strip0 + nstrips (p is the GLOBAL strip index)
    if ((uint64_t)c->tagbase + (uint64_t)strip_first + (uint64_t)s.nstrips * nbl + 2u >= 0xFFFFFFF0ull) {
        NW_HIP_TRY(hipMemsetAsync(c->gran, 0, c->gran_cap, (hipStream_t)stream));
        c->tagbase = 1;
    }
    const int64_t qlen = nw::rowpack_len((int32_t)s.nblocks);
    if ((st = grow((void **)&c->rowpack, &c->rowpack_cap, (size_t)qlen * 16 * nbl)) != NW_OK) return st;
    if ((st = grow((void **)&c->scratch, &c->scratch_cap, (size_t)s.waves * nw::kScratchWords * 4)) != NW_OK)
        return st;

    // per-launch control words: reset, keeping a failure not yet reported (nw_link.hip nw_ctrl_reset)
    if (nw::launch_ctrl_reset(c->ctrl, stream) != hipSuccess) return NW_ERR_HIP;
    const uint8_t *s1u = n1 > 0 ? (const uint8_t *)d_s1 : (const uint8_t *)c->ctrl;
    const uint8_t *s2u = n2 > 0 ? (const uint8_t *)d_s2 : (const uint8_t *)c->ctrl;
    // v_perm score tables when every substitution score minus 2*GAP fits int8
    // (the kernel falls back to compares on the device when s1 holds more than
    // kMaxPerm distinct characters).
    // table bytes are s - 2 GAP in the w form (NW, and SW in the strips), s - GAP
    // for SW in the panels (the u form)
    const int32_t off = sw && panels ? p->gap : 2 * p->gap;
    const bool perm_ok = fits_i8(p->match - off) && fits_i8(p->mismatch - off) &&
                         !(p->flags & NW_FLAG_NO_PROFILE);
    if (sw) {
        // per-strip best cells (zeroed on the launch stream) + best / key words
        const size_t need = (size_t)(s.nstrips + 8) * sizeof(int32_t);
        if ((st = grow((void **)&c->smax, &c->smax_cap, need)) != NW_OK) return st;
        NW_HIP_TRY(hipMemsetAsync(c->smax, 0, (size_t)(s.nstrips + 8) * sizeof(int32_t), (hipStream_t)stream));
    }
    for (int32_t b = 0; b < nbl; ++b)  // (block b's side characters: s2 + b * n2)
        if (nw::launch_rowpack(s1u, n1, s2u + (n2 > 0 ? (int64_t)b * n2 : 0), n2, 0, perm_ok ? 1 : 0, c->meta,
                               (char *)c->rowpack + (int64_t)b * qlen * 16, qlen, stream) != hipSuccess)
            return NW_ERR_HIP;

    nw::FillArgs a;
    std::memset(&a, 0, sizeof a);
    a.table = d_t - start;  // table + c = global column c (start = 0 but for column bands)
    a.pitch = pitch;
    a.col_end = start + pitch;
    a.strip0 = (int32_t)strip_first;
    a.feed_in = cb ? cb->feed_in : nullptr;
    a.feed_out = cb ? cb->feed_out : nullptr;
    a.feed_tag = cb ? cb->tag : 0u;
    a.rowpack = c->rowpack;
    a.s1 = n1 > 0 ? (const uint8_t *)d_s1 : (const uint8_t *)c->ctrl;
    a.n1 = n1;
    a.n2 = n2;
    a.row0 = 0;
    a.col0 = col0;
    a.nstrips = (int32_t)s.nstrips;
    a.nblocks = (int32_t)s.nblocks;
    a.gran = c->gran;
    a.gstride = s.gstride;
    a.M = (int32_t)s.M;
    a.tagbase = c->tagbase;
    a.ctrl = c->ctrl;
    a.halo_in = band ? band->halo_in : nullptr;
    a.halo_out = band ? band->halo_out : nullptr;
    a.halo_tag = band ? band->tag : 0u;
    a.scratch = c->scratch;
    a.perm = perm_ok ? 1 : 0;
    a.charmap = c->meta;
    a.nprof = (const uint32_t *)(c->meta + 256);
    a.trace = c->trace;
    a.match = p->match;
    a.mismatch = p->mismatch;
    a.gap = p->gap;
    a.flags = p->flags;
    // s_memrealtime runs at 100 MHz: 100000 ticks per ms
    a.timeout_ticks = (uint64_t)(p->timeout_ms > 0 ? p->timeout_ms : 20000) * 100000ull;
    a.sw = sw ? 1 : 0;
    a.smax = sw ? c->smax : nullptr;
    a.nbl = nbl;
    a.hin0 = cy ? cy->hin_first : 1;
    a.hoshift = cy ? cy->hout_shift : 0;
    a.tstride = cy ? cy->t_stride : 0;
    a.qstride = qlen * 16;
    a.hstride = n1 + 1;
    if ((panels ? nw::launch_panels(a, s.K, s.NC, (int)s.waves, stream)
                : nw::launch_fill(a, s.K, s.NC, (int)s.waves, stream)) != hipSuccess)
        return NW_ERR_HIP;
    // a column band's local column 0 (band r-1's last column) from its feed
    if (cb && cb->feed_in &&
        nw::launch_colband_edge(cb->feed_in, d_t, pitch, n2, p->gap, start, stream) != hipSuccess)
        return NW_ERR_HIP;
    c->tagbase += (uint32_t)(strip_first + s.nstrips * nbl) + 1u;
    c->last_waves = (int)s.waves;
    c->last_strips = (int)s.nstrips;
    c->last_sub = s.K;
    c->last_nc = s.NC;
    c->last_col0 = (int)col0;
    c->last_kernel = s.kernel;
    if (sw) {
        // best cell: max over the strips, then the first row-major cell holding it
        if (!c->swinfo) NW_HIP_TRY(hipMalloc(&c->swinfo, 16 * sizeof(int64_t)));  // [0..9] traceback info, [12] locate key
        int32_t *best = c->smax + s.nstrips;
        uint64_t *key = (uint64_t *)(c->swinfo + 12);
        // (TIMING_ONLY: the strips stored into a scratch tile and the caller's table
        // was never written, so there is no corner to fix up in it)
        if (half && !(p->flags & NW_FLAG_TIMING_ONLY) && nw::launch_sw_fixup(d_t, pitch, n1, n2, (const uint8_t *)d_s1, (const uint8_t *)d_s2, p->match,
                                        p->mismatch, p->gap, col0, (int32_t)(nw::kWave * s.K * s.NC), c->smax,
                                        stream) != hipSuccess)
            return NW_ERR_HIP;
        if (nw::launch_sw_locate(d_t, pitch, n1, n2, col0, (int32_t)(nw::kWave * s.K * s.NC), c->smax,
                                 (int32_t)s.nstrips, key, best, stream) != hipSuccess)
            return NW_ERR_HIP;
    }
    return NW_OK;
}

int nw_fill_device_async(nw_ctx *c, const int8_t *d_s1, int64_t n1, const int8_t *d_s2,
                         int64_t n2, const nw_params *p, int32_t *d_t, int64_t pitch,
                         void *stream) {
    return launch_fill(c, d_s1, n1, d_s2, n2, p, nullptr, nullptr, d_t, pitch, stream);
}

int nw_fill_band_async(nw_ctx *c, const int8_t *d_s1, int64_t n1, const int8_t *d_s2_band,
                       int64_t n2_band, const nw_params *p, const nw_band *band, int32_t *d_t,
                       int64_t pitch, void *stream) {
    if (!band) return NW_ERR_ARG;
    return launch_fill(c, d_s1, n1, d_s2_band, n2_band, p, band, nullptr, d_t, pitch, stream);
}

int nw_fill_band_cycle_async(nw_ctx *c, const int8_t *d_s1, int64_t n1, const int8_t *d_s2_blocks,
                             int64_t n2_blk, const nw_params *p, const nw_band_cycle *cy, int32_t *d_t,
                             int64_t pitch, void *stream) {
    if (!cy) return NW_ERR_ARG;
    return launch_fill(c, d_s1, n1, d_s2_blocks, n2_blk, p, nullptr, nullptr, d_t, pitch, stream, cy);
}

void nw_band_layout(int64_t n2, int32_t nbands, int32_t r, int64_t *n_rows, int64_t *start) {
    // mpi-horz-driver.cpp:31-32 / mpi-horz.cpp:16: base = (n2+1)/P rows per band; bands
    // after the first carry one extra (halo) row; the last band takes the remainder.
    int64_t rows = 0, st = 0;
    if (nbands > 0 && r >= 0 && r < nbands) {
        const int64_t total = n2 + 1, base = total / nbands;
        rows = base + (r > 0 ? 1 : 0) + (r == nbands - 1 ? total % nbands : 0);
        st = base * r - (r > 0 ? 1 : 0);
    }
    if (n_rows) *n_rows = rows;
    if (start) *start = st;
}

// A halo / feed buffer: its own allocation (so that HIP IPC exports exactly it),
// fine-grained -- the producing kernel on ANOTHER GPU writes it over xGMI with
// system-scope stores while this GPU's kernel polls it with system-scope loads,
// and system-scope coherence between agents is what fine-grained memory gives
// (coarse-grained memory is only coherent at agent scope).
// NW_LINK_COARSE=1 (diagnostics, one device and one process only): plain
// coarse-grained memory, to tell the feed's uncached-memory cost from the
// protocol's.  Coarse-grained memory is coherent at agent
// scope only, so such a buffer is never exported (nw_ipc_get_handle refuses).
static bool link_coarse() {
    static const bool coarse = [] {
        const char *e = std::getenv("NW_LINK_COARSE");
        const bool on = e != nullptr && e[0] == '1';
        if (on)
            std::fprintf(stderr, "libnwhip: NW_LINK_COARSE=1: halo / feed / link buffers are coarse-grained "
                                 "(single-device diagnostics; IPC export refused)\n");
        return on;
    }();
    return coarse;
}

static hipError_t alloc_link_buffer(void **p, size_t bytes) {
    if (link_coarse()) return hipMalloc(p, bytes);
    return hipExtMallocWithFlags(p, bytes, hipDeviceMallocFinegrained);
}

int nw_colband_layout(int64_t n1, int64_t n2, int32_t nbands, int32_t r, const nw_params *p,
                      int64_t *strip_first, int64_t *strip_count, int64_t *start, int64_t *n_cols) {
    int64_t sf = 0, sc = 0, st = 0, nc = 0;
    const int rc = colband_layout(n1, n2, nbands, r, p, 256, &sf, &sc, &st, &nc);
    if (strip_first) *strip_first = sf;
    if (strip_count) *strip_count = sc;
    if (start) *start = st;
    if (n_cols) *n_cols = nc;
    return rc;
}

int nw_fill_colband_async(nw_ctx *c, const int8_t *d_s1, int64_t n1, const int8_t *d_s2, int64_t n2,
                          const nw_params *p, const nw_colband *band, int32_t *d_t, int64_t pitch,
                          void *stream) {
    if (!band) return NW_ERR_ARG;
    return launch_fill(c, d_s1, n1, d_s2, n2, p, nullptr, band, d_t, pitch, stream);
}

// Row band in horizontal strips: the (4, 1) strip kernel on the TRANSPOSED band
// (the NW table of (s2_band, s1) is the band's transpose, the scores being
// symmetric), in global row numbers: its "columns" are global rows row0 + 1 ..
// row0 + R (strips of 256 rows from row0 + 1), its "rows" the band's columns
// 0..n1; the store waves write the row-major band table (store_strip_tr).
static constexpr int kTbandLeadSleep = 8;

int nw_fill_tband_async(nw_ctx *c, const int8_t *d_s1, int64_t n1, const int8_t *d_s2, int64_t R,
                        const nw_params *p, const nw_tband *tb, int32_t *d_t, int64_t pitch, void *stream) {
    if (!c || !d_t || !tb || !d_s1 || !d_s2 || n1 < 1 || R < 1 || n1 >= INT32_MAX || R >= INT32_MAX ||
        tb->row0 < 0 || tb->row0 + R >= INT32_MAX)
        return NW_ERR_ARG;
    if (!valid_params(p)) return NW_ERR_ARG;
    // shapes: (4, 1) (the default) or (2, 2) -- 256-row strips either way
    if (p->mode != NW_MODE_NW || p->kernel == NW_KERNEL_PANELS) return NW_ERR_UNSUPPORTED;
    int tC = 4, tNC = 1;
    if (p->substrips != 0 || p->strip_waves != 0) {
        tC = p->substrips ? p->substrips : 4;
        tNC = p->strip_waves ? p->strip_waves : 1;
        if (!((tC == 4 && tNC == 1) || (tC == 2 && tNC == 2))) return NW_ERR_UNSUPPORTED;
    }
    if (tb->tag == 0 || (((uintptr_t)tb->feed_in | (uintptr_t)tb->feed_out) & 7u) != 0) return NW_ERR_ARG;
    if ((tb->flags & ~(uint32_t)NW_TBAND_DENSE_POLLS) != 0) return NW_ERR_ARG;
    if ((tb->row0 > 0) != (tb->feed_in != nullptr)) return NW_ERR_ARG;
    if (tb->feed_out && (p->flags & 1)) return NW_ERR_ARG;  // needs the real last row
    if ((p->flags & NW_FLAG_DEBUG_NO_CHAIN) && (tb->feed_in || tb->feed_out)) return NW_ERR_ARG;  // (no fill to hand on)
    if ((((uintptr_t)d_t + 4u) & 255u) != 0 || pitch % nw::kWave != 0 || pitch < n1 + 4) return NW_ERR_ARG;
    {  // |w| bound of launch_fill, with the global row
        const long long m = std::max({std::llabs(p->match), std::llabs(p->mismatch), std::llabs(p->gap)});
        if ((m + std::llabs(p->gap)) * (long long)(n1 + tb->row0 + R + 2) >= (1LL << 28)) return NW_ERR_ARG;
    }
    NW_HIP_TRY(hipSetDevice(c->device));
    // the transposed band: R + 1 "columns" (global rows row0 .. row0 + R, the first
    // one the feed), n1 + 1 "rows" (the band's columns)
    Shape s = make_shape(R, n1, p->waves, tC, tNC, c->cus, 1, false, NW_KERNEL_STRIPS);
    if (!shape_valid(s) || s.nstrips > INT32_MAX / 2 || s.nblocks > INT32_MAX / 2) return NW_ERR_ARG;
    // Leftover rows: when the band's last strip would run ALONE as one more pass over
    // all n1 columns (strips = k * workers + 1, e.g. config 4's last band: 65537 rows =
    // 257 strips on 256 CUs), its rows are computed by the row-scan finisher after the
    // strips instead (nw_finish.hip: one prefix-max scan per row across the width).
    int64_t Rs = R, L = 0;
    if (s.nstrips > s.waves && (s.nstrips - 1) % s.waves == 0 && !(p->flags & NW_FLAG_NO_FINISH) &&
        !(p->flags & 1)) {
        L = R - 256 * (s.nstrips - 1);
        Rs = R - L;
        s = make_shape(Rs, n1, p->waves, tC, tNC, c->cus, 1, false, NW_KERNEL_STRIPS);
        if (!shape_valid(s)) return NW_ERR_ARG;
    }
    int st;
    const size_t gran_need = (size_t)(s.M * s.gstride) * sizeof(uint64_t);
    bool fresh = false;
    if ((st = grow((void **)&c->gran, &c->gran_cap, gran_need, &fresh)) != NW_OK) return st;
    if (fresh) {
        NW_HIP_TRY(hipMemsetAsync(c->gran, 0, c->gran_cap, (hipStream_t)stream));
        c->tagbase = 1;
    }
    if ((uint64_t)c->tagbase + (uint64_t)s.nstrips + 2u >= 0xFFFFFFF0ull) {
        NW_HIP_TRY(hipMemsetAsync(c->gran, 0, c->gran_cap, (hipStream_t)stream));
        c->tagbase = 1;
    }
    const int64_t qlen = nw::rowpack_len((int32_t)s.nblocks);
    if ((st = grow((void **)&c->rowpack, &c->rowpack_cap, (size_t)qlen * 16)) != NW_OK) return st;
    if ((st = grow((void **)&c->scratch, &c->scratch_cap, (size_t)s.waves * nw::kScratchWords * 4)) != NW_OK)
        return st;
    // per-launch control words: reset, keeping a failure not yet reported (nw_link.hip nw_ctrl_reset)
    if (nw::launch_ctrl_reset(c->ctrl, stream) != hipSuccess) return NW_ERR_HIP;
    const bool perm_ok = fits_i8(p->match - 2 * p->gap) && fits_i8(p->mismatch - 2 * p->gap) &&
                         !(p->flags & NW_FLAG_NO_PROFILE);
    // lanes carry the band's row characters (charmap of s2_band), the row packs the columns' (s1)
    if (nw::launch_rowpack((const uint8_t *)d_s2, R, (const uint8_t *)d_s1, n1, 0, perm_ok ? 1 : 0, c->meta,
                           c->rowpack, qlen, stream) != hipSuccess)
        return NW_ERR_HIP;
    nw::FillArgs a;
    std::memset(&a, 0, sizeof a);
    a.table = d_t;
    a.pitch = pitch;
    a.col_end = INT64_MAX;
    a.strip0 = 0;
    a.feed_in = tb->feed_in;
    a.feed_out = L > 0 ? nullptr : tb->feed_out;  // (with a finisher, it publishes the last row)
    a.feed_tag = tb->tag;
    a.rowpack = c->rowpack;
    a.s1 = (const uint8_t *)d_s2 - tb->row0;  // s1[y - 1] = global row y's character
    a.n1 = tb->row0 + Rs;                     // global last row the strips sweep
    a.n2 = n1;
    a.row0 = 0;
    a.col0 = tb->row0 + 1;                    // first swept global row
    a.nstrips = (int32_t)s.nstrips;
    a.nblocks = (int32_t)s.nblocks;
    a.gran = c->gran;
    a.gstride = s.gstride;
    a.M = (int32_t)s.M;
    a.tagbase = c->tagbase;
    a.ctrl = c->ctrl;
    a.scratch = c->scratch;
    a.perm = perm_ok ? 1 : 0;
    a.charmap = c->meta;
    a.nprof = (const uint32_t *)(c->meta + 256);
    a.trace = c->trace;
    a.match = p->match;
    a.mismatch = p->mismatch;
    a.gap = p->gap;
    a.flags = p->flags;
    a.timeout_ticks = (uint64_t)(p->timeout_ms > 0 ? p->timeout_ms : 20000) * 100000ull;
    a.nbl = 1;
    a.hin0 = 1;
    a.qstride = qlen * 16;
    a.hstride = n1 + 1;
    a.tr = 1;
    a.tr_y0 = tb->row0;
    a.tr_pub = (int32_t)(Rs - 1 - 256 * (s.nstrips - 1));  // the last row's column in the last strip
    {
        static const int compute_pub = [] {
            const char *e = std::getenv("NW_TR_PUB_COMPUTE");
            return e != nullptr && e[0] == '1';
        }();
        a.tr_store_pub = compute_pub && tNC == 1 ? 0 : 1;  // ((2, 2): the store waves publish)
        // With sparse polls the band's unfed leading strip (band 0's strip 0: the whole
        // chain's leader) sleeps 8 x 64 clocks per 64-step iteration (~8 %): followers that
        // run 1-2 % slower for a while then keep up instead of delaying every strip below
        // them (mean strip-to-strip lag 16.3-17.4 -> 12.5 us, leader 25.8 -> 27.0-28.0 ms;
        // profiles/r06f_lead_sleep.txt).  Dense polls slow the leader by themselves and
        // need no throttle (lag 10.0 us at a leader of 28.0-28.5 ms with none, 29.7-29.8
        // with 8: profiles/r06n_lead_dense.txt).  NW_LEAD_SLEEP overrides both (A/B).
        a.tr_dense = (tb->flags & NW_TBAND_DENSE_POLLS) != 0 ? 1 : 0;
        static const int lead_env = [] {
            const char *e = std::getenv("NW_LEAD_SLEEP");
            return e != nullptr ? std::atoi(e) : -1;
        }();
        a.lead_sleep = lead_env >= 0 ? lead_env : tNC != 1 ? 0 : a.tr_dense ? 0 : kTbandLeadSleep;
    }
    if (nw::launch_fill(a, tC, tNC, (int)s.waves, stream) != hipSuccess) return NW_ERR_HIP;
    if (nw::launch_tband_edges(tb->feed_in, d_t, pitch, n1, R + 1, p->gap, tb->row0, stream) != hipSuccess)
        return NW_ERR_HIP;
    c->tagbase += (uint32_t)s.nstrips + 1u;
    c->last_finish_rows = (int)L;
    if (L > 0) {
        nw::FinishArgs f;
        std::memset(&f, 0, sizeof f);
        f.chunk_cols = nw::finish_chunk_cols(n1, c->cus);
        // debug (tests): NW_DEBUG_FINISH_WIDE=1 forces the 8192-column chunks (K = 32),
        // otherwise only chosen above 8 chunks per CU (~4.2M columns on 256 CUs)
        if (const char *e = std::getenv("NW_DEBUG_FINISH_WIDE")) {
            if (e[0] == '1') f.chunk_cols = nw::finish_chunk_cols(INT64_MAX / 4, c->cus);
        }
        f.nchunks = (int32_t)((n1 + f.chunk_cols - 1) / f.chunk_cols);
        const size_t need = (size_t)L * (size_t)f.nchunks * sizeof(uint64_t);
        bool fresh = false;
        if ((st = grow((void **)&c->look, &c->look_cap, need, &fresh)) != NW_OK) return st;
        if (fresh || (uint64_t)c->look_tag + 2u * (uint64_t)L + 2u >= 0xFFFFFFF0ull) {
            NW_HIP_TRY(hipMemsetAsync(c->look, 0, c->look_cap, (hipStream_t)stream));
            c->look_tag = 1;
        }
        f.table = d_t;
        f.pitch = pitch;
        f.s1 = (const uint8_t *)d_s1;
        f.n1 = n1;
        f.s2 = (const uint8_t *)d_s2;
        f.li0 = Rs + 1;
        f.nrows = L;
        f.grow0 = tb->row0;
        f.match = p->match;
        f.mismatch = p->mismatch;
        f.gap = p->gap;
        f.look = c->look;
        f.tag0 = c->look_tag;
        f.ctrl = c->ctrl;
        f.feed_out = tb->feed_out;
        f.feed_tag = tb->tag;
        f.timeout_ticks = a.timeout_ticks;
        if (nw::launch_finish_rows(f, stream) != hipSuccess) return NW_ERR_HIP;
        c->look_tag += 2u * (uint32_t)L + 2u;
    }
    c->last_waves = (int)s.waves;
    c->last_strips = (int)s.nstrips;
    c->last_sub = 4;
    c->last_nc = 1;
    c->last_col0 = 1;
    c->last_kernel = NW_KERNEL_STRIPS;
    return NW_OK;
}

int64_t nw_feed_bytes(int64_t n2) {
    return n2 < 0 ? 0 : round_up(n2 + 1, nw::kWave) * (int64_t)sizeof(uint64_t);
}

int nw_feed_alloc(int device, int64_t n2, uint64_t **d_feed) {
    if (!d_feed || n2 < 0) return NW_ERR_ARG;
    *d_feed = nullptr;
    if (device >= 0) NW_HIP_TRY(hipSetDevice(device));
    void *q = nullptr;
    const size_t bytes = (size_t)nw_feed_bytes(n2);
    hipError_t e = alloc_link_buffer(&q, bytes);
    if (e != hipSuccess) return e == hipErrorOutOfMemory ? NW_ERR_OOM : NW_ERR_HIP;
    if (hipMemset(q, 0, bytes) != hipSuccess) {
        (void)hipFree(q);
        return NW_ERR_HIP;
    }
    *d_feed = (uint64_t *)q;
    return NW_OK;
}

int64_t nw_halo_bytes(int64_t n1) { return n1 < 0 ? 0 : (n1 + 1) * (int64_t)sizeof(uint64_t); }

int nw_halo_alloc(int device, int64_t n1, uint64_t **d_halo) { return nw_halo_alloc_regions(device, n1, 1, d_halo); }

int nw_halo_alloc_regions(int device, int64_t n1, int32_t nregions, uint64_t **d_halo) {
    if (!d_halo || n1 < 0 || nregions < 1) return NW_ERR_ARG;
    *d_halo = nullptr;
    if (device >= 0) NW_HIP_TRY(hipSetDevice(device));
    void *p = nullptr;
    const size_t bytes = (size_t)nw_halo_bytes(n1) * (size_t)nregions;
    hipError_t e = alloc_link_buffer(&p, bytes);
    if (e != hipSuccess) return e == hipErrorOutOfMemory ? NW_ERR_OOM : NW_ERR_HIP;
    if (hipMemset(p, 0, bytes) != hipSuccess) {
        (void)hipFree(p);
        return NW_ERR_HIP;
    }
    *d_halo = (uint64_t *)p;
    return NW_OK;
}

int nw_halo_free(uint64_t *d_halo) {
    if (!d_halo) return NW_ERR_ARG;
    NW_HIP_TRY(hipFree(d_halo));
    return NW_OK;
}

int nw_link_alloc(int device, uint32_t **d_word) {
    if (!d_word) return NW_ERR_ARG;
    *d_word = nullptr;
    if (device >= 0) NW_HIP_TRY(hipSetDevice(device));
    void *q = nullptr;
    hipError_t e = alloc_link_buffer(&q, 256);
    if (e != hipSuccess) return e == hipErrorOutOfMemory ? NW_ERR_OOM : NW_ERR_HIP;
    if (hipMemset(q, 0, 256) != hipSuccess) {
        (void)hipFree(q);
        return NW_ERR_HIP;
    }
    *d_word = (uint32_t *)q;
    return NW_OK;
}

int nw_link_wait_async(uint32_t *d_word, uint32_t value, int32_t timeout_ms, void *stream) {
    return nw_link_wait_ctx_async(nullptr, d_word, value, timeout_ms, stream);
}

int nw_link_wait_ctx_async(nw_ctx *c, uint32_t *d_word, uint32_t value, int32_t timeout_ms, void *stream) {
    if (!d_word || timeout_ms < 0) return NW_ERR_ARG;
    const uint64_t ticks = (uint64_t)(timeout_ms > 0 ? timeout_ms : 20000) * 100000ull;
    return nw::launch_link_wait(d_word, value, ticks, c ? c->ctrl : nullptr, stream) == hipSuccess ? NW_OK
                                                                                                  : NW_ERR_HIP;
}

int nw_link_signal_async(uint32_t *d_word, uint32_t value, void *stream) {
    if (!d_word) return NW_ERR_ARG;
    return nw::launch_link_signal(d_word, value, stream) == hipSuccess ? NW_OK : NW_ERR_HIP;
}

int nw_link_status(const uint32_t *d_word, uint32_t *out) {
    if (!d_word || !out) return NW_ERR_ARG;
    NW_HIP_TRY(hipMemcpy(out, d_word + 1, sizeof(uint32_t), hipMemcpyDeviceToHost));
    return NW_OK;
}

int nw_ipc_get_handle(const void *d_ptr, void *handle) {
    if (!d_ptr || !handle) return NW_ERR_ARG;
    if (link_coarse()) return NW_ERR_UNSUPPORTED;  // (a peer would see stale data)
    hipIpcMemHandle_t h;
    NW_HIP_TRY(hipIpcGetMemHandle(&h, const_cast<void *>(d_ptr)));
    std::memcpy(handle, &h, sizeof h < NW_IPC_HANDLE_BYTES ? sizeof h : NW_IPC_HANDLE_BYTES);
    return NW_OK;
}

int nw_ipc_open_handle(const void *handle, void **d_ptr) {
    if (!handle || !d_ptr) return NW_ERR_ARG;
    hipIpcMemHandle_t h;
    std::memset(&h, 0, sizeof h);
    std::memcpy(&h, handle, sizeof h < NW_IPC_HANDLE_BYTES ? sizeof h : NW_IPC_HANDLE_BYTES);
    NW_HIP_TRY(hipIpcOpenMemHandle(d_ptr, h, hipIpcMemLazyEnablePeerAccess));
    return NW_OK;
}

int nw_ipc_close_handle(void *d_ptr) {
    if (!d_ptr) return NW_ERR_ARG;
    NW_HIP_TRY(hipIpcCloseMemHandle(d_ptr));
    return NW_OK;
}

int nw_ctx_status(nw_ctx *c, void *stream) {
    if (!c) return NW_ERR_ARG;
    NW_HIP_TRY(hipSetDevice(c->device));
    uint32_t w[nw::kCtrlWords] = {};
    NW_HIP_TRY(hipMemcpyAsync(w, c->ctrl, sizeof w, hipMemcpyDeviceToHost, (hipStream_t)stream));
    NW_HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    // the last launch's error word, or a failure any earlier launch (or a link wait)
    // recorded since the last read -- read and cleared (nw_link.hip nw_ctrl_reset)
    const bool failed = (w[1] != 0 && w[13] == 0) || w[8] != 0;
    if (w[8] != 0 || w[12] != 0) {
        for (int k = 0; k < 5; ++k) c->last_failure[k] = w[8 + k];
        // the last launch (poisoned by the folded failure, or failed on its own) is
        // not folded into [12] until the next reset: count it here
        if (w[1] != 0 && w[13] == 0) c->last_failure[4] = w[12] + 1;
    } else if (w[1] != 0 && w[13] == 0) {  // the last launch failed (not folded in yet)
        c->last_failure[0] = w[1];
        c->last_failure[1] = w[2];
        c->last_failure[2] = w[3];
        c->last_failure[3] = w[4];
        c->last_failure[4] = 1;
    }
    if (failed) {
        // clear the record and mark the last launch's words as read (ctrl[13])
        static const uint32_t cleared[nw::kCtrlWords - 8] = {0, 0, 0, 0, 0, 1, 0, 0};
        NW_HIP_TRY(hipMemcpyAsync(c->ctrl + 8, cleared, sizeof cleared, hipMemcpyHostToDevice, (hipStream_t)stream));
        NW_HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    }
    return failed ? NW_ERR_TIMEOUT : NW_OK;
}

int nw_fill_device(nw_ctx *c, const int8_t *d_s1, int64_t n1, const int8_t *d_s2, int64_t n2,
                   const nw_params *p, int32_t *d_t, int64_t pitch, void *stream,
                   nw_result *out) {
    if (!c) return NW_ERR_ARG;
    NW_HIP_TRY(hipSetDevice(c->device));
    if (out) NW_HIP_TRY(hipEventRecord(c->ev0, (hipStream_t)stream));
    int st = nw_fill_device_async(c, d_s1, n1, d_s2, n2, p, d_t, pitch, stream);
    if (st != NW_OK || !out) return st;
    NW_HIP_TRY(hipEventRecord(c->ev1, (hipStream_t)stream));
    st = nw_ctx_status(c, stream);
    std::memset(out, 0, sizeof *out);
    out->status = st;
    float ms = 0.f;
    NW_HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    out->kernel_ms = ms;
    out->cells = n1 * n2;
    out->table_bytes = (double)(n1 + 1) * (double)(n2 + 1) * 4.0;
    out->strips = c->last_strips;
    out->waves = c->last_waves;
    out->substrips = c->last_sub;
    out->strip_waves = c->last_nc;
    out->kernel = c->last_kernel;
    int32_t score = 0;
    if (p->mode == NW_MODE_SW) {
        // best cell (nw_sw.hip locate): score and its first row-major position
        uint64_t key = 0;
        NW_HIP_TRY(hipMemcpy(&score, c->smax + c->last_strips, 4, hipMemcpyDeviceToHost));
        NW_HIP_TRY(hipMemcpy(&key, c->swinfo + 12, 8, hipMemcpyDeviceToHost));
        out->end_i = score > 0 ? (int64_t)(key >> 32) : 0;
        out->end_j = score > 0 ? (int64_t)(key & 0xFFFFFFFFull) : 0;
    } else {
        NW_HIP_TRY(hipMemcpy(&score, d_t + n2 * pitch + n1, 4, hipMemcpyDeviceToHost));
        out->end_i = n2;
        out->end_j = n1;
    }
    out->score = score;
    return st;
}

int nw_sw_traceback(nw_ctx *c, const int8_t *d_s1, int64_t n1, const int8_t *d_s2, int64_t n2,
                    const nw_params *p, const int32_t *d_t, int64_t pitch, int64_t end_i, int64_t end_j,
                    uint8_t *host_ops, int64_t ops_cap, nw_alignment *out) {
    if (!c || !d_t || !p || !out || n1 < 0 || n2 < 0 || end_i < 0 || end_j < 0 || end_i > n2 || end_j > n1)
        return NW_ERR_ARG;
    if ((end_j > 0 && !d_s1) || (end_i > 0 && !d_s2) || (ops_cap > 0 && !host_ops) || ops_cap < 0)
        return NW_ERR_ARG;
    if (!valid_params(p) || p->mode != NW_MODE_SW) return NW_ERR_ARG;
    NW_HIP_TRY(hipSetDevice(c->device));
    // the table may have been filled on any stream (nw_fill_device_async on a
    // non-blocking stream has no ordering with the null stream used below)
    NW_HIP_TRY(hipDeviceSynchronize());
    int st;
    const size_t need = (size_t)std::max<int64_t>(end_i + end_j + 1, 1);
    if ((st = grow((void **)&c->ops, &c->ops_cap, need)) != NW_OK) return st;
    // window geometry: band half-width and windows per round (NW_TB_BAND /
    // NW_TB_MAXWIN override them: narrow bands and short rounds for the tests)
    int32_t band = nw::kTbBandDefault, maxwin = nw::kTbMaxWinDefault;
    if (const char *e = std::getenv("NW_TB_BAND")) band = std::max(1, std::min(256, std::atoi(e)));
    if (const char *e = std::getenv("NW_TB_MAXWIN")) maxwin = std::max(1, std::atoi(e));
    maxwin = (int32_t)std::min<int64_t>(maxwin, end_i / 64 + 1);
    if ((st = grow((void **)&c->tbscratch, &c->tbscratch_cap, nw::sw_tb_scratch_bytes(maxwin, band))) != NW_OK)
        return st;
    NW_HIP_TRY(hipEventRecord(c->ev0, nullptr));
    int64_t info[10];
    const int he = nw::run_sw_traceback(d_t, pitch, n1, (const uint8_t *)d_s1, (const uint8_t *)d_s2, p->match,
                                        p->mismatch, p->gap, end_i, end_j, c->ops, (int64_t)need, c->tbscratch,
                                        maxwin, band, info, nullptr);
    if (he != hipSuccess) {
        std::fprintf(stderr, "libnwhip: SW traceback failed: %s\n", hipGetErrorString((hipError_t)he));
        return NW_ERR_HIP;
    }
    NW_HIP_TRY(hipEventRecord(c->ev1, nullptr));
    NW_HIP_TRY(hipEventSynchronize(c->ev1));
    if (std::getenv("NW_TB_DEBUG"))
        std::fprintf(stderr, "nw_sw_traceback: %lld moves, %lld rounds, %lld windows (band %d)\n", (long long)info[0],
                     (long long)info[4], (long long)info[5], band);
    float ms = 0.f;
    NW_HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    std::memset(out, 0, sizeof *out);
    out->end_i = end_i;
    out->end_j = end_j;
    out->n_ops = info[0];
    out->begin_i = info[1];
    out->begin_j = info[2];
    out->traceback_ms = ms;
    out->status = info[3] == 0 ? NW_OK : NW_ERR_HIP;
    NW_HIP_TRY(hipMemcpy(&out->score, d_t + end_i * pitch + end_j, 4, hipMemcpyDeviceToHost));
    if (info[3] != 0) return out->status;
    if (info[0] > ops_cap) return NW_ERR_ARG;
    if (info[0] > 0) {
        // the kernel walks end -> begin; hand the ops over begin -> end
        NW_HIP_TRY(hipMemcpy(host_ops, c->ops, (size_t)info[0], hipMemcpyDeviceToHost));
        std::reverse(host_ops, host_ops + info[0]);
    }
    return NW_OK;
}

// ---- host-buffer entry points (the drop-in path) ----------------------------
//
// One HostPath per device, created on first use and kept: the context, the
// device table and sequence buffers (grow-only: a caller looping over pairs pays
// no hipMalloc / hipFree of the table per call), a non-blocking copy stream and
// two pinned staging chunks.  The table comes back to the caller's (pageable)
// buffer through the staging chunks: DMA of chunk k+1 overlaps the threaded
// memcpy of chunk k into the caller's rows (tools/d2h_bench.cpp measured the
// alternatives; DESIGN.md "drop-in path").  nw_host_release frees it all.
namespace {

struct HostPath {
    std::mutex mu;
    nw_ctx *c = nullptr;
    int32_t *tab = nullptr;  // 256-byte aligned allocation; the table starts nw_table_offset() in
    size_t tab_cap = 0;
    int8_t *s1 = nullptr, *s2 = nullptr;
    size_t s1_cap = 0, s2_cap = 0;
    char *stage[3] = {nullptr, nullptr, nullptr};
    size_t stage_cap = 0;  // bytes per staging chunk
    hipStream_t copy = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
};
constexpr int kStages = 3;

// staging chunk: up to 256 MiB (a third of the table, at least 16 MiB), pinned
// with hipHostMallocCoherent (tools/d2h_bench.cpp on the box: 40 GB through 3 x
// 256 MiB coherent chunks and 8 copy threads at 56.6 GB/s, the bare pinned
// hipMemcpy2D's 56.4; 128 MiB default-flag chunks 45-53)
constexpr size_t kStageMax = 256u << 20, kStageMin = 16u << 20;
// tables up to this size stay cached between calls; a larger one is released
// when its call returns (it would crowd out the caller's own device work)
constexpr size_t kKeepTableBytes = 16ull << 30;
HostPath g_host[64];

void host_trim(HostPath &h) {
    if (h.tab && h.tab_cap > kKeepTableBytes) {
        (void)hipFree(h.tab);
        h.tab = nullptr;
        h.tab_cap = 0;
    }
}

void host_free(HostPath &h) {
    if (h.c) (void)hipSetDevice(h.c->device);
    if (h.tab) (void)hipFree(h.tab);
    if (h.s1) (void)hipFree(h.s1);
    if (h.s2) (void)hipFree(h.s2);
    for (int k = 0; k < kStages; ++k) {
        if (h.stage[k]) (void)hipHostFree(h.stage[k]);
        if (h.ev[k]) (void)hipEventDestroy(h.ev[k]);
        h.stage[k] = nullptr;
        h.ev[k] = nullptr;
    }
    h.stage_cap = 0;
    if (h.copy) (void)hipStreamDestroy(h.copy);
    nw_ctx_destroy(h.c);
    h.c = nullptr;
    h.tab = nullptr;
    h.s1 = h.s2 = nullptr;
    h.tab_cap = h.s1_cap = h.s2_cap = 0;
    h.copy = nullptr;
}

// Device and sequence buffers for an n1 x n2 table; copies s1 / s2 in.
int host_prepare(HostPath &h, int dev, const int8_t *s1, int64_t n1, const int8_t *s2, int64_t n2,
                 int32_t **d_t, int64_t *pitch) {
    int st;
    if (!h.c && (st = nw_ctx_create(dev, &h.c)) != NW_OK) return st;
    NW_HIP_TRY(hipSetDevice(dev));
    *pitch = nw_table_pitch(n1);
    // column 1 on a 256-byte line: the allocation (256-byte aligned) + nw_table_offset
    const size_t need = (size_t)nw_table_bytes(n1, n2) + 256;
    if (need > h.tab_cap) {  // (grow drops the old buffer first: one table at a time)
        if ((st = grow((void **)&h.tab, &h.tab_cap, need)) != NW_OK) return st;
    }
    if ((st = grow((void **)&h.s1, &h.s1_cap, (size_t)std::max<int64_t>(n1, 1))) != NW_OK) return st;
    if ((st = grow((void **)&h.s2, &h.s2_cap, (size_t)std::max<int64_t>(n2, 1))) != NW_OK) return st;
    if (n1 > 0) NW_HIP_TRY(hipMemcpy(h.s1, s1, (size_t)n1, hipMemcpyHostToDevice));
    if (n2 > 0) NW_HIP_TRY(hipMemcpy(h.s2, s2, (size_t)n2, hipMemcpyHostToDevice));
    *d_t = h.tab + (n1 >= 1 ? nw_table_offset() : 0);  // (no column 1 when n1 = 0)
    return NW_OK;
}

void par_memcpy(char *dst, const char *src, size_t bytes, int threads) {
    if (threads <= 1 || bytes < (8u << 20)) {
        std::memcpy(dst, src, bytes);
        return;
    }
    std::vector<std::thread> ts;
    const size_t per = (bytes / (size_t)threads + 4095) & ~(size_t)4095;
    for (int t = 1; t < threads; ++t) {
        const size_t o = (size_t)t * per;
        if (o >= bytes) break;
        ts.emplace_back([=] { std::memcpy(dst + o, src + o, std::min(per, bytes - o)); });
    }
    std::memcpy(dst, src, std::min(per, bytes));
    for (auto &t : ts) t.join();
}

int copy_threads() {
    if (const char *e = std::getenv("NW_COPY_THREADS")) return std::max(1, std::atoi(e));
    return (int)std::min<unsigned>(8u, std::max(1u, std::thread::hardware_concurrency()));
}

// Rows 0..n2 (n1 + 1 int32 each) of the device table into host rows of
// `stride` int32 (the reference layout: stride = n1 + 1), through the pinned
// staging chunks.
int host_staging(HostPath &h, size_t table_bytes) {
    size_t want = std::min(kStageMax, std::max(kStageMin, (table_bytes / kStages + (2u << 20) - 1) & ~((size_t)(2u << 20) - 1)));
    if (want > h.stage_cap) {
        for (int k = 0; k < kStages; ++k) {
            if (h.stage[k]) (void)hipHostFree(h.stage[k]);
            h.stage[k] = nullptr;
        }
        h.stage_cap = 0;
        for (int k = 0; k < kStages; ++k)
            NW_HIP_TRY(hipHostMalloc((void **)&h.stage[k], want, hipHostMallocCoherent));
        h.stage_cap = want;
    }
    for (int k = 0; k < kStages; ++k)
        if (!h.ev[k]) NW_HIP_TRY(hipEventCreateWithFlags(&h.ev[k], hipEventDisableTiming));
    if (!h.copy) NW_HIP_TRY(hipStreamCreateWithFlags(&h.copy, hipStreamNonBlocking));
    return NW_OK;
}

int host_copy_back(HostPath &h, const int32_t *d_t, int64_t pitch, int64_t n1, int64_t n2, int32_t *host,
                   int64_t stride) {
    int st;
    const size_t w = (size_t)(n1 + 1) * 4;
    const int64_t rows = n2 + 1;
    if ((st = host_staging(h, w * (size_t)rows)) != NW_OK) return st;
    const int64_t rpc = std::max<int64_t>(1, (int64_t)(h.stage_cap / w));
    if ((size_t)rpc * w > h.stage_cap) {  // one row wider than a chunk: direct
        NW_HIP_TRY(hipMemcpy2D(host, (size_t)stride * 4, d_t, (size_t)pitch * 4, w, (size_t)rows,
                               hipMemcpyDeviceToHost));
        return NW_OK;
    }
    const int64_t nch = (rows + rpc - 1) / rpc;
    const int threads = copy_threads();
    auto issue = [&](int64_t ch) -> hipError_t {
        const int64_t r0 = ch * rpc, nr = std::min(rpc, rows - r0);
        hipError_t e = hipMemcpy2DAsync(h.stage[ch % kStages], w, d_t + r0 * pitch, (size_t)pitch * 4, w,
                                        (size_t)nr, hipMemcpyDeviceToHost, h.copy);
        return e == hipSuccess ? hipEventRecord(h.ev[ch % kStages], h.copy) : e;
    };
    // the fill ran on the null stream (synchronous), so the copy stream sees the table
    for (int64_t ch = 0; ch < std::min<int64_t>(kStages, nch); ++ch) NW_HIP_TRY(issue(ch));
    double t_dma = 0, t_cpy = 0;
    auto tnow = [] { return std::chrono::steady_clock::now(); };
    auto sec = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
    for (int64_t ch = 0; ch < nch; ++ch) {
        const auto a0 = tnow();
        NW_HIP_TRY(hipEventSynchronize(h.ev[ch % kStages]));
        const auto a1 = tnow();
        t_dma += sec(a0, a1);
        const int64_t r0 = ch * rpc, nr = std::min(rpc, rows - r0);
        const char *src = h.stage[ch % kStages];
        if (stride * 4 == (int64_t)w) {
            par_memcpy((char *)(host + r0 * stride), src, (size_t)nr * w, threads);
        } else {
            for (int64_t r = 0; r < nr; ++r) std::memcpy(host + (r0 + r) * stride, src + (size_t)r * w, w);
        }
        t_cpy += sec(a1, tnow());
        if (ch + kStages < nch) NW_HIP_TRY(issue(ch + kStages));
    }
    if (std::getenv("NW_HOST_TIMING"))
        std::fprintf(stderr, "  copy back: %lld chunks of %zu MiB, %d threads: waiting on DMA %.1f ms, copying %.1f ms\n",
                     (long long)nch, h.stage_cap >> 20, threads, t_dma * 1e3, t_cpy * 1e3);
    return NW_OK;
}

int host_device(const nw_params *p, int *dev) {
    *dev = p->device;
    if (*dev < 0 && hipGetDevice(dev) != hipSuccess) return NW_ERR_NODEVICE;
    if (*dev < 0 || *dev >= 64) return NW_ERR_ARG;
    return NW_OK;
}

}  // namespace

int nw_host_warmup(int device) {
    int dev = device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return NW_ERR_NODEVICE;
    if (dev < 0 || dev >= 64) return NW_ERR_ARG;
    HostPath &h = g_host[dev];
    std::lock_guard<std::mutex> lock(h.mu);
    int st;
    if (!h.c && (st = nw_ctx_create(dev, &h.c)) != NW_OK) return st;
    NW_HIP_TRY(hipSetDevice(dev));
    return host_staging(h, kStageMax * kStages);
}

void nw_host_release(int device) {
    for (int d = 0; d < 64; ++d) {
        if (device >= 0 && d != device) continue;
        std::lock_guard<std::mutex> lock(g_host[d].mu);
        host_free(g_host[d]);
    }
}

int nw_sw_align(const int8_t *s1, int64_t n1, const int8_t *s2, int64_t n2, const nw_params *p,
                uint8_t *host_ops, int64_t ops_cap, nw_alignment *out) {
    if (!p || p->mode != NW_MODE_SW || !out || n1 < 0 || n2 < 0 || (n1 > 0 && !s1) || (n2 > 0 && !s2))
        return NW_ERR_ARG;
    int dev, st;
    if ((st = host_device(p, &dev)) != NW_OK) return st;
    HostPath &h = g_host[dev];
    std::lock_guard<std::mutex> lock(h.mu);
    int32_t *d_t = nullptr;
    int64_t pitch = 0;
    nw_result r;
    std::memset(&r, 0, sizeof r);
    st = host_prepare(h, dev, s1, n1, s2, n2, &d_t, &pitch);
    if (st == NW_OK) st = nw_fill_device(h.c, h.s1, n1, h.s2, n2, p, d_t, pitch, nullptr, &r);
    if (st == NW_OK) st = nw_sw_traceback(h.c, h.s1, n1, h.s2, n2, p, d_t, pitch, r.end_i, r.end_j, host_ops,
                                          ops_cap, out);
    if (st == NW_OK) out->fill_ms = r.kernel_ms;
    host_trim(h);
    out->status = st;
    return st;
}

int nw_fill(const int8_t *s1, int64_t n1, const int8_t *s2, int64_t n2, const nw_params *p,
            int32_t *host_t, nw_result *out) {
    nw_params def;
    if (!p) {
        nw_params_default(&def);
        p = &def;
    }
    if (n1 < 0 || n2 < 0 || (n1 > 0 && !s1) || (n2 > 0 && !s2)) return NW_ERR_ARG;
    int dev, st;
    if ((st = host_device(p, &dev)) != NW_OK) return st;
    HostPath &h = g_host[dev];
    std::lock_guard<std::mutex> lock(h.mu);
    int32_t *d_t = nullptr;
    int64_t pitch = 0;
    nw_result r;
    std::memset(&r, 0, sizeof r);
    const auto t0 = std::chrono::steady_clock::now();
    st = host_prepare(h, dev, s1, n1, s2, n2, &d_t, &pitch);
    const auto t1 = std::chrono::steady_clock::now();
    if (st == NW_OK) st = nw_fill_device(h.c, h.s1, n1, h.s2, n2, p, d_t, pitch, nullptr, &r);
    const auto t2 = std::chrono::steady_clock::now();
    if (st == NW_OK && host_t) st = host_copy_back(h, d_t, pitch, n1, n2, host_t, n1 + 1);
    const auto t3 = std::chrono::steady_clock::now();
    if (std::getenv("NW_HOST_TIMING")) {
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::fprintf(stderr, "nw_fill: prepare (context, buffers, H2D) %.1f ms, fill %.1f ms (kernel %.1f), "
                     "copy back %.1f ms (%.1f GB/s)\n", ms(t0, t1), ms(t1, t2), r.kernel_ms, ms(t2, t3),
                     host_t ? (double)(n1 + 1) * (n2 + 1) * 4 / (ms(t2, t3) * 1e6) : 0.0);
    }
    host_trim(h);
    r.status = st;
    if (out) *out = r;
    return st;
}

int nw_fill_emb(const int8_t *s1, int64_t n1, const int8_t *s2, int64_t n2, const nw_params *p,
                int32_t *host_t, nw_result *out) {
    // The emb layout of src/idxarray/idxarray-emb-mt.cpp:7-37 / src/common/driver2.cpp:20-22:
    // nCols = n1 + 2; column 0 holds each row's progress counter, which the reference
    // fill leaves at its final value nCols (:49, the row loop's `int& j`, and :36 for
    // row 0); columns 1 .. n1+1 hold the serial table.  Fill as nw_fill, copy the
    // table into columns 1.., then write column 0.
    nw_params def;
    if (!p) {
        nw_params_default(&def);
        p = &def;
    }
    if (!host_t || n1 < 0 || n2 < 0 || (n1 > 0 && !s1) || (n2 > 0 && !s2)) return NW_ERR_ARG;
    int dev, st;
    if ((st = host_device(p, &dev)) != NW_OK) return st;
    HostPath &h = g_host[dev];
    std::lock_guard<std::mutex> lock(h.mu);
    int32_t *d_t = nullptr;
    int64_t pitch = 0;
    nw_result r;
    std::memset(&r, 0, sizeof r);
    st = host_prepare(h, dev, s1, n1, s2, n2, &d_t, &pitch);
    if (st == NW_OK) st = nw_fill_device(h.c, h.s1, n1, h.s2, n2, p, d_t, pitch, nullptr, &r);
    if (st == NW_OK) st = host_copy_back(h, d_t, pitch, n1, n2, host_t + 1, n1 + 2);
    if (st == NW_OK)
        for (int64_t i = 0; i <= n2; ++i) host_t[i * (n1 + 2)] = (int32_t)(n1 + 2);
    host_trim(h);
    r.status = st;
    if (out) *out = r;
    return st;
}

// Debug hook: the control words of the last launch (ticket, error code, watchdog
// site / need / seen -- nw_fill.hip give_up); include/nw_hip.h documents them.
int nw_debug_ctrl(nw_ctx *c, uint32_t *out8) {
    if (!c || !out8) return NW_ERR_ARG;
    NW_HIP_TRY(hipSetDevice(c->device));
    NW_HIP_TRY(hipDeviceSynchronize());
    NW_HIP_TRY(hipMemcpy(out8, c->ctrl, 32, hipMemcpyDeviceToHost));
    return NW_OK;
}

// Debug hook: the first failure recorded since the status before last was read
// (code, site word, need, seen, failed launches) -- what nw_ctx_status cleared
// when it last reported NW_ERR_TIMEOUT -- or, before any such read, the live words.
int nw_debug_failure(nw_ctx *c, uint32_t *out5) {
    if (!c || !out5) return NW_ERR_ARG;
    NW_HIP_TRY(hipSetDevice(c->device));
    NW_HIP_TRY(hipDeviceSynchronize());
    uint32_t w[nw::kCtrlWords] = {};
    NW_HIP_TRY(hipMemcpy(w, c->ctrl, sizeof w, hipMemcpyDeviceToHost));
    if (w[8] != 0 || w[12] != 0) {
        for (int k = 0; k < 5; ++k) out5[k] = w[8 + k];
        if (w[1] != 0 && w[13] == 0) out5[4] = w[12] + 1;  // + the last launch (nw_ctx_status)
    } else
        for (int k = 0; k < 5; ++k) out5[k] = c->last_failure[k];
    return NW_OK;
}

// Debug hook: per-strip trace buffer, device memory of at least
// strips * nw_debug_trace_words() uint64 (see nwhip.Context.set_trace); NULL = off.
int nw_debug_set_trace(nw_ctx *c, void *d_trace) {
    if (!c) return NW_ERR_ARG;
    c->trace = (uint64_t *)d_trace;
    return NW_OK;
}

int32_t nw_debug_trace_words(void) { return nw::kTraceWords; }

void nw_tuned_shape(int64_t n1, int64_t n2, int32_t *substrips, int32_t *strip_waves) {
    int32_t c = 2, nc = 2;
    if (n1 >= 0 && n2 >= 0) tuned_shape(n1, n2, &c, &nc);
    if (substrips) *substrips = c;
    if (strip_waves) *strip_waves = nc;
}

void nw_auto_shape(int64_t n1, int64_t n2, int32_t cus, int32_t *kernel, int32_t *substrips, int32_t *strip_waves) {
    int32_t k = NW_KERNEL_STRIPS, c = 2, nc = 2;
    if (n1 >= 0 && n2 >= 0) tuned_shape(n1, n2, &c, &nc, &k, std::max(cus, 1));
    if (kernel) *kernel = k;
    if (substrips) *substrips = c;
    if (strip_waves) *strip_waves = nc;
}

}  // extern "C"
