// nw_strips_2x4.hip -- the strip kernel (nw_strips.h) for C = 2 columns per
// lane and NC = 4 compute waves per strip: 512-column strips on half-word rings
// (Lay::kHalf), Smith-Waterman only.
#include "nw_strips.h"

namespace nw {
#if !defined(NW_ONLY_C) || (NW_ONLY_C == 2 && NW_ONLY_NC == 4)
void launch_strips_2x4(const FillArgs &a, int grid, hipStream_t s) { launch_c<2, 4>(a, grid, s); }
#else
void launch_strips_2x4(const FillArgs &, int, hipStream_t) {}
#endif
}  // namespace nw
