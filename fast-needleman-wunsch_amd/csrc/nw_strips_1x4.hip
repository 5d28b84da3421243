// nw_strips_1x4.hip -- the strip kernel (nw_strips.h) for C = 1 columns per
// lane and NC = 4 compute waves per strip (one shape per TU: parallel builds).
#include "nw_strips.h"

namespace nw {
#if !defined(NW_ONLY_C) || (NW_ONLY_C == 1 && NW_ONLY_NC == 4)
void launch_strips_1x4(const FillArgs &a, int grid, hipStream_t s) { launch_c<1, 4>(a, grid, s); }
#else
void launch_strips_1x4(const FillArgs &, int, hipStream_t) {}
#endif
}  // namespace nw
