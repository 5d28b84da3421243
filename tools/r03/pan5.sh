#!/bin/bash
# panel kernel: left values loaded after the group (NW_ROWS_LATEFEED) vs before: parity, A/B, trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03u
mkdir -p $O
cd $R
B=$R/fast-needleman-wunsch_amd/build
NWHIP_LIB=$B/libnwhip_late.so timeout -k 10 400 python3 -u -m pytest tests/test_panels.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/panels_late_tests.txt 2>&1 || exit 1
for i in 1 2; do
  for v in "" _late; do
    echo "lib$v" >> $O/pan_ab3.txt
    NWHIP_LIB=$B/libnwhip$v.so timeout -k 10 300 python3 -u tools/quick_time.py --sizes 262144 --kernel 2 --reps 4 >> $O/pan_ab3.txt 2>&1 || exit 2
  done
done
NWHIP_LIB=$B/libnwhip_late.so timeout -k 10 300 python3 -u tools/panel_trace.py > $O/pan_trace3.txt 2>&1 || exit 3
