#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03z
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_bands.py tests/test_tbands.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/twoproc.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/twoproc.txt; exit $rc
