// nw_fill.hip -- the strip kernel's host-side dispatch (one TU per shape:
// nw_strips_<C>x<NC>.hip, device code in nw_strips.h) and the small kernels
// around every fill: the column-character map, the row packs, the column-band
// edge.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "nw_dev.h"
#include "nw_internal.h"
#include "nw_strips.h"  // (Lay<>, sw_shape: layouts only, no kernel instantiated here)

namespace nw {
// Column-character map of a launch, in two kernels: nw_charmap_scan (a grid of
// workgroups, each byte of s1 read once, coalesced) ORs which byte values occur
// in s1 into present[8]; nw_charmap_finish (one workgroup) turns that into
// charmap[c] = index of c among them in increasing order (0xFF: absent) and
// *nprof = how many distinct characters s1 holds, then zeroes present[] for the
// next launch (it starts zeroed: nw_ctx_create).
constexpr int kScanBytesPerWG = 8192;
__global__ __launch_bounds__(256) void nw_charmap_scan(const uint8_t *__restrict__ s1, int64_t n1,
                                                        uint32_t *__restrict__ present) {
    __shared__ uint32_t loc[8];
    if (threadIdx.x < 8) loc[threadIdx.x] = 0;
    __syncthreads();
    uint32_t mine[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n1; i += stride) {
        const uint32_t c = s1[i];
#pragma unroll
        for (int w = 0; w < 8; ++w) mine[w] |= (c >> 5) == (uint32_t)w ? 1u << (c & 31) : 0u;
    }
#pragma unroll
    for (int w = 0; w < 8; ++w)
        if (mine[w]) atomicOr(&loc[w], mine[w]);
    __syncthreads();
    if (threadIdx.x < 8 && loc[threadIdx.x]) atomicOr(present + threadIdx.x, loc[threadIdx.x]);
}

__global__ __launch_bounds__(256) void nw_charmap_finish(uint32_t *__restrict__ present,
                                                          uint8_t *__restrict__ charmap,
                                                          uint32_t *__restrict__ nprof) {
    __shared__ uint32_t pw[8], before[8];
    if (threadIdx.x < 8) pw[threadIdx.x] = present[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int w = 0; w < 8; ++w) {
            before[w] = acc;
            acc += (uint32_t)__builtin_popcount(pw[w]);
        }
        *nprof = acc;
    }
    __syncthreads();
    const uint32_t c = threadIdx.x, w = c >> 5, bit = 1u << (c & 31);
    const uint32_t idx = before[w] + (uint32_t)__builtin_popcount(pw[w] & (bit - 1u));
    charmap[c] = (pw[w] & bit) != 0u ? (uint8_t)min(idx, 255u) : (uint8_t)0xFF;
    if (threadIdx.x < 8) present[threadIdx.x] = 0u;
}

// rowpack16[idx] = B[x .. x+15] (16 bytes), x = idx - kQOff, B[y] = s2[row0 + y - 1]
// for 1 <= y <= n2 (local rows of this launch), else 0.  With `perm` set and
// at most kMaxPerm distinct column characters (*nprof, from nw_charmap) the
// bytes are MAPPED: charmap[B[y]], or 7 for a character in no column (and for
// rows outside 1..n2) -- the SUB_PERM selector bytes.
__global__ void nw_rowpack(const uint8_t *__restrict__ s2, int64_t n2, int64_t row0,
                           const uint8_t *__restrict__ charmap, const uint32_t *__restrict__ nprof,
                           int32_t perm, u32x4 *__restrict__ q, int64_t qlen) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= qlen) return;
    const bool map = perm != 0 && *nprof <= kMaxPerm;
    const int64_t x = idx - kQOff;
    u32x4 v = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int64_t y = x + k;
        uint32_t b = (y >= 1 && y <= n2) ? (uint32_t)s2[row0 + y - 1] : 0u;
        if (map) b = (y >= 1 && y <= n2) ? min((uint32_t)charmap[b], 7u) : 7u;
        v[k >> 2] |= b << (8 * (k & 3));
    }
    q[idx] = v;
}

// Column band: local column 0 of the band's table = the left band's last column,
// from the feed granules (w form) this launch consumed -- all of them, so their
// values are final; system-scope loads as in the kernel (peer-written memory).
__global__ __launch_bounds__(256) void nw_colband_edge(const uint64_t *__restrict__ feed,
                                                       int32_t *__restrict__ table, int64_t pitch,
                                                       int64_t n2, int32_t gap, int64_t start) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i > n2) return;
    const uint64_t g = __hip_atomic_load(feed + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    table[i * pitch] = (int32_t)((int64_t)(int32_t)(uint32_t)g + (int64_t)gap * (i + start));
}

int launch_colband_edge(const uint64_t *feed, int32_t *table, int64_t pitch, int64_t n2, int32_t gap,
                        int64_t start, void *stream) {
    const int64_t rows = n2 + 1;
    hipLaunchKernelGGL(nw_colband_edge, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       feed, table, pitch, n2, gap, start);
    return (int)hipGetLastError();
}

// Row band in horizontal strips: the edges the strips do not sweep.  Row 0 is
// the previous band's last row (the feed the launch consumed, w form in global
// coordinates: t = w + gap * (x + start)) or, for the first band, the boundary
// t[0][x] = x * gap (serial.cpp:16); column 0 of rows 1 .. rows-1 is the
// boundary t[y][0] = (start + y) * gap (serial.cpp:17), start = global row of
// the band's row 0.
__global__ __launch_bounds__(256) void nw_tband_edges(const uint64_t *__restrict__ feed,
                                                      int32_t *__restrict__ table, int64_t pitch, int64_t n1,
                                                      int64_t rows, int32_t gap, int64_t start) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i <= n1) {
        int64_t v = (int64_t)gap * i;
        if (feed != nullptr) {
            const uint64_t g = __hip_atomic_load(feed + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            v = (int64_t)(int32_t)(uint32_t)g + (int64_t)gap * (i + start);
        }
        table[i] = (int32_t)v;
    }
    if (i >= 1 && i < rows) table[i * pitch] = (int32_t)((int64_t)gap * (start + i));
}

int launch_tband_edges(const uint64_t *feed, int32_t *table, int64_t pitch, int64_t n1, int64_t rows,
                       int32_t gap, int64_t start, void *stream) {
    const int64_t n = std::max<int64_t>(n1 + 1, rows);
    hipLaunchKernelGGL(nw_tband_edges, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       feed, table, pitch, n1, rows, gap, start);
    return (int)hipGetLastError();
}

// entries of 16 bytes: iteration j <= nblocks + 3 (prefetch of the last one)
// reads up to index kQOff + 64 * (nblocks + 3) + 48
int64_t rowpack_len(int32_t nblocks) { return kQOff + 64 * ((int64_t)nblocks + 4) + 16; }

int launch_rowpack(const uint8_t *d_s1, int64_t n1, const uint8_t *d_s2, int64_t n2, int64_t row0,
                   int32_t perm, uint8_t *meta, void *d_q, int64_t qlen, void *stream) {
    uint8_t *charmap = meta;
    uint32_t *nprof = (uint32_t *)(meta + 256);
    uint32_t *present = (uint32_t *)(meta + 272);
    const int64_t g = std::min<int64_t>(256, std::max<int64_t>(1, (n1 + kScanBytesPerWG - 1) / kScanBytesPerWG));
    hipLaunchKernelGGL(nw_charmap_scan, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, d_s1, n1, present);
    hipLaunchKernelGGL(nw_charmap_finish, dim3(1), dim3(256), 0, (hipStream_t)stream, present, charmap, nprof);
    const int bs = 256;
    const int64_t nb = (qlen + bs - 1) / bs;
    hipLaunchKernelGGL(nw_rowpack, dim3((unsigned)nb), dim3(bs), 0, (hipStream_t)stream, d_s2, n2,
                       row0, charmap, nprof, perm, (u32x4 *)d_q, qlen);
    return (int)hipGetLastError();
}

// Supported (columns per lane, compute waves per strip) shapes, one TU each
// (nw_strips_<C>x<NC>.hip).  Experiment builds (make variant DEFS="-DNW_ONLY_C=2
// -DNW_ONLY_NC=2") instantiate one strip shape only.
#ifdef NW_ONLY_C
#define NW_SHAPE(c, nc) ((c) == NW_ONLY_C && (nc) == NW_ONLY_NC)
#else
#define NW_SHAPE(c, nc) true
#endif
#define NW_DECL(c, nc) void launch_strips_##c##x##nc(const FillArgs &a, int grid, hipStream_t s);
NW_DECL(4, 1) NW_DECL(2, 1) NW_DECL(1, 1) NW_DECL(2, 2) NW_DECL(1, 2) NW_DECL(1, 4) NW_DECL(2, 4)
#undef NW_DECL

bool shape_ok(int substrips, int strip_waves) {
#ifdef NW_ONLY_C
    if (substrips != NW_ONLY_C || strip_waves != NW_ONLY_NC) return false;
#endif
    switch (substrips * 8 + strip_waves) {
        case 4 * 8 + 1: case 2 * 8 + 1: case 1 * 8 + 1:
        case 2 * 8 + 2: case 1 * 8 + 2: case 1 * 8 + 4:
        case 2 * 8 + 4:  // (half-word rings: Smith-Waterman only, sw_shape_ok / launch_fill)
            return true;
        default:
            return false;
    }
}

bool sw_shape_ok(int substrips, int strip_waves) {
    return shape_ok(substrips, strip_waves) && sw_shape(substrips, strip_waves);
}

int launch_fill(const FillArgs &a, int substrips, int strip_waves, int grid, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (!shape_ok(substrips, strip_waves)) return (int)hipErrorInvalidValue;
    if (Lay<2, 4>::kHalf && substrips == 2 && strip_waves == 4 && !a.sw) return (int)hipErrorInvalidValue;
    switch (substrips * 8 + strip_waves) {
#define NW_CASE(c, nc) \
        case c * 8 + nc: if constexpr (NW_SHAPE(c, nc)) launch_strips_##c##x##nc(a, grid, s); break;
        NW_CASE(4, 1) NW_CASE(2, 1) NW_CASE(1, 1) NW_CASE(2, 2) NW_CASE(1, 2) NW_CASE(1, 4) NW_CASE(2, 4)
#undef NW_CASE
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

int lds_bytes(int substrips, int strip_waves) {
    switch (substrips * 8 + strip_waves) {
        case 4 * 8 + 1: return Lay<4, 1>::kBytes;
        case 2 * 8 + 1: return Lay<2, 1>::kBytes;
        case 1 * 8 + 1: return Lay<1, 1>::kBytes;
        case 2 * 8 + 2: return Lay<2, 2>::kBytes;
        case 1 * 8 + 2: return Lay<1, 2>::kBytes;
        case 2 * 8 + 4: return Lay<2, 4>::kBytes;
        default: return Lay<1, 4>::kBytes;
    }
}

const char *kernel_variant() { return "strips(NCx64xC, compute+store waves, diag ring 128, vperm, gran16, w form; 2x4 half-word SW rings) + panels(row scan 4x256, feeder-in/out waves)"; }

}  // namespace nw
