#!/bin/bash
# first GPU contact of the row-scan panel kernel: ubench, parity, timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
timeout -k 10 120 tools/ubench/rowscan > $O/rowscan.txt 2>&1 || exit 2
timeout -k 10 600 python3 -u -m pytest tests/test_panels.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/panels_tests.txt 2>&1
echo "pytest rc=$?" >> $O/panels_tests.txt
timeout -k 10 300 python3 -u tools/quick_time.py --sizes 262144 --kernel 2 --shapes 4:4,2:8 --flags 0 --reps 2 > $O/panels_time.txt 2>&1 || exit 4
timeout -k 10 300 python3 -u tools/quick_time.py --sizes 262144 --kernel 2 --shapes 4:4,2:8 --flags 8 --reps 2 >> $O/panels_time.txt 2>&1 || exit 5
timeout -k 10 300 python3 -u tools/quick_time.py --sizes 262144 --kernel 1 --shapes 1:4 --flags 0 --reps 2 >> $O/panels_time.txt 2>&1 || exit 6
timeout -k 10 300 python3 -u tools/quick_time.py --sizes 65536,32768 --kernel 2 --shapes 4:1,2:2,1:4,2:4 --reps 2 >> $O/panels_time.txt 2>&1 || exit 7
echo done >> $O/panels_time.txt
