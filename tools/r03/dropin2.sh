#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
G=tests/golden/bdna
for rep in 1 2 3; do
  NW_HOST_TIMING=1 timeout -k 10 300 fast-needleman-wunsch_amd/build/nw_driver $G/big1.bdna $G/big2.bdna >> $O/dropin2.txt 2>&1 || exit 3
  NW_COPY_THREADS=16 NW_HOST_TIMING=1 timeout -k 10 300 fast-needleman-wunsch_amd/build/nw_driver $G/big1.bdna $G/big2.bdna >> $O/dropin2.txt 2>&1 || exit 3
done
timeout -k 10 300 tools/d2h_bench 100000 8 256 1 >> $O/dropin2.txt 2>&1 || exit 4
