#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03h
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/tband_trace.py --n2 1024,16384,65536 > $O/tband_trace.txt 2>&1
