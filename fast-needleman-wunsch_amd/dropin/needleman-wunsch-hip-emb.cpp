// needleman-wunsch-hip-emb.cpp -- the MI355X fill plugin for the reference's
// "emb" callers (src/common/driver2.cpp, src/idxarray/idxarray-emb-mt.cpp):
// same symbol `void needlemanWunsch(dnaArray, dnaArray, int*)`, but the caller's
// table has n1+2 columns, column 0 being a per-row progress counter that the
// reference fill leaves at n1+2 (idxarray-emb-mt.cpp:49) and columns 1.. the
// serial values.  Failures exit with status 2 (the contract has no error
// channel), as in needleman-wunsch-hip.cpp.
#include <cstdio>
#include <cstdlib>

#include "nw_dropin.hpp"
#include "nw_hip.h"

namespace {
// device context created at plugin load (see needleman-wunsch-hip.cpp)
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
    const int st = nw_fill_emb(s1.dna, s1.size, s2.dna, s2.size, &p, (int32_t *)t, nullptr);
    if (st != NW_OK) {
        std::fprintf(stderr, "needlemanWunsch (libnwhip, emb layout): %s\n", nw_strerror(st));
        std::exit(2);
    }
}
