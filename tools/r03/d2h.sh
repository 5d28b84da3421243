#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
for th in 8 16; do
  timeout -k 10 300 tools/d2h_bench 100000 $th 256 1 >> $O/d2h2.txt 2>&1 || exit 3
done
