#!/bin/bash
# block-cyclic bands parity first (new kernel path), then the whole GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03c
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_cycles.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/cycles.txt 2>&1 || exit 1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.txt 2>&1 || exit 2
