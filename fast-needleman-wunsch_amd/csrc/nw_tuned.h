// nw_tuned.h -- kernel family and shape per table size for auto fills (nw_params
// kernel = substrips = strip_waves = 0).  Written by tools/tune.py from measurements on
// an MI355X (AMD Radeon Graphics; tools/tune_table.json); entries in increasing
// min_cells, the last one that applies wins.
#pragma once

namespace nw {
struct TunedShape {
    double min_cells;  // (n1 + 1) * (n2 + 1) at least
    int kernel;        // 1 = strips (nw_fill.hip), 2 = panels (nw_rows.hip)
    int c, nc;         // columns per lane, chained compute waves per strip / panel
};
constexpr TunedShape kTuned[] = {
    {0.0, 1, 4, 1},  // best at 4096^2: 47 GCUPS
    {67129345.0, 1, 2, 2},  // best at 16384^2: 211 GCUPS
    {536920065.0, 1, 2, 2},  // best at 32768^2: 421 GCUPS
    {2147581953.0, 1, 2, 2},  // best at 65536^2: 760 GCUPS
    {8590131201.0, 2, 2, 4},  // best at 131072^2: 1052 GCUPS
    {34360131585.0, 2, 4, 4},  // best at 262144^2: 1534 GCUPS
};
}  // namespace nw
