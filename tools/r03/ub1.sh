#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03u
mkdir -p $O
cd $R
timeout -k 10 200 tools/ubench/panel_store 64 0,4,16 0 > $O/panel_store.txt 2>&1
