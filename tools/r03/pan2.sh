#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03u
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/panel_trace.py > $O/pan_trace.txt 2>&1
