#!/bin/bash
# horizontal-strip row bands: parity tests, then the per-GPU band geometry timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03h
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_tbands.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tbands.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tbands.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/tband_time.py > $O/tband_time.txt 2>&1 || exit 31
timeout -k 10 300 python3 -u tools/tband_time.py --flags 8 --vertical "" >> $O/tband_time.txt 2>&1 || exit 32
timeout -k 10 300 python3 -u tools/tband_time.py --n1 262144 --n2 262144 --vertical 1:4 >> $O/tband_time.txt 2>&1 || exit 33
