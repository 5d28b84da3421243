#!/bin/bash
# panel kernel at 256k: full fill, stores to scratch (no HBM), no store waves; the store pattern alone
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03u
mkdir -p $O
cd $R
for f in 0 1 8; do
  timeout -k 10 300 python3 -u tools/quick_time.py --sizes 262144 --kernel 2 --flags $f --reps 3 >> $O/pan_flags.txt 2>&1 || exit 31
done
timeout -k 10 200 tools/ubench/panel_store 64 0,4 0 >> $O/pan_flags.txt 2>&1
