// nw_strips_2x1.hip -- the strip kernel (nw_strips.h) for C = 2 columns per
// lane and NC = 1 compute waves per strip (one shape per TU: parallel builds).
#include "nw_strips.h"

namespace nw {
#if !defined(NW_ONLY_C) || (NW_ONLY_C == 2 && NW_ONLY_NC == 1)
void launch_strips_2x1(const FillArgs &a, int grid, hipStream_t s) { launch_c<2, 1>(a, grid, s); }
#else
void launch_strips_2x1(const FillArgs &, int, hipStream_t) {}
#endif
}  // namespace nw
