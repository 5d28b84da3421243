#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03u
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/trace_strips.py --n 262144 --sub 1 --nc 4 > $O/clk.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/trace_strips.py --n 262144 --sub 1 --nc 4 --flags 1 >> $O/clk.txt 2>&1 || exit 2
