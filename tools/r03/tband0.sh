#!/bin/bash
# horizontal-strip row bands: parity tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03h
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_tbands.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tbands.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tbands.txt; exit $rc
