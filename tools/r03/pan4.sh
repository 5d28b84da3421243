#!/bin/bash
# panel kernel with vector-loaded row characters: panel parity, prefetch distance 1/2/3, trace, bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03u
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_panels.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/panels_tests.txt 2>&1 || exit 1
B=$R/fast-needleman-wunsch_amd/build
for i in 1 2; do
  for v in "" _wpd1 _wpd3; do
    echo "lib$v" >> $O/pan_ab2.txt
    NWHIP_LIB=$B/libnwhip$v.so timeout -k 10 300 python3 -u tools/quick_time.py --sizes 262144 --kernel 2 --reps 4 >> $O/pan_ab2.txt 2>&1 || exit 2
  done
done
timeout -k 10 300 python3 -u tools/panel_trace.py > $O/pan_trace2.txt 2>&1 || exit 3
timeout -k 10 300 python3 -u bench.py > $O/bench2.json 2> $O/bench2.err || exit 4
