// needleman-wunsch-hip.cpp -- the MI355X fill plugin.
//
// Defines the reference plugin symbol `void needlemanWunsch(dnaArray, dnaArray,
// int*)` (serial.cpp:4 / sentinel-mt.cpp:4 / idxarray-mt.cpp:4) and forwards to
// the C ABI of libnwhip.so.  Like the reference fills it writes every cell of the
// caller-owned table `t` ((s2.size+1) x (s1.size+1) int32, row-major,
// serial.cpp:6-7) and returns nothing.  Unlike them it can fail (no device, OOM):
// the reference contract has no error channel (driver.cpp:28), so a failure is
// reported on stderr and the process exits with status 2 -- loudly, never with
// a silently wrong or CPU-computed table.
//
// By default the device context (HIP runtime, copy stream, pinned staging) is
// created by the first call, so the caller's timer around needlemanWunsch
// (driver.cpp:26-30) sees the whole cost, as it does for the reference fills.
// NW_WARM_START=1 creates it when the plugin is loaded instead -- a static
// initializer, before the caller's main(), the way a resident service holds it
// -- so that the timer sees the fill and the table's transfer only (INTEGRATION.md
// reports both).  A failure there is ignored: the call reports it.
#include <cstdio>
#include <cstdlib>

#include "nw_dropin.hpp"
#include "nw_hip.h"

namespace {
struct Warmup {
    Warmup() {
        const char *e = std::getenv("NW_WARM_START");
        if (e != nullptr && e[0] == '1') (void)nw_host_warmup(-1);
    }
} g_warmup;
}  // namespace

void needlemanWunsch(dnaArray s1, dnaArray s2, int *t) {
    nw_params p;
    nw_params_default(&p);
    p.match = NW_MATCH;
    p.mismatch = NW_MISMATCH;
    p.gap = NW_GAP;
    nw_result r;
    const int st = nw_fill(s1.dna, s1.size, s2.dna, s2.size, &p, (int32_t *)t, &r);
    if (st != NW_OK) {
        std::fprintf(stderr, "needlemanWunsch (libnwhip): %s\n", nw_strerror(st));
        std::exit(2);
    }
    if (std::getenv("NW_VERBOSE"))
        std::fprintf(stderr, "libnwhip: kernel %.3f ms, %.2f GCUPS, %d strips, %d waves\n",
                     r.kernel_ms, r.kernel_ms > 0 ? r.cells / (r.kernel_ms * 1e6) : 0.0, r.strips,
                     r.waves);
}
