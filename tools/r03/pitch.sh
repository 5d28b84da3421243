#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
for sl in 64 0 128 256 512 1024 2048 4096; do
  timeout -k 10 120 tools/ubench/panel_store $sl 0,40,256 0 >> $O/pitch.txt 2>&1 || exit 3
done
echo done >> $O/pitch.txt
