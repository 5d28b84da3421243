#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03z
mkdir -p $O
cd $R
NW_LINK_COARSE=1 timeout -k 10 300 python3 -u tools/local_bands_time.py > $O/local_h_coarse.txt 2>&1 || exit 1
