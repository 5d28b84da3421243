#!/bin/bash
# round-3 baseline diagnostics on one box: the row-scan ubench, the 256k fill
# per shape with the debug flags (0 = normal, 8 = compute waves only, 1 =
# stores to a scratch tile), and the two band geometries of the multi-GPU model
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
timeout -k 10 120 tools/ubench/rowscan > $O/rowscan.txt 2>&1 || exit 2
for f in 0 8 1; do
  timeout -k 10 240 python3 -u tools/quick_time.py --sizes 262144 --shapes 1:4,4:1,2:2 --flags $f --reps 2 >> $O/diag0.txt 2>&1 || exit 3
done
timeout -k 10 240 python3 -u tools/rect_time.py --n1 65536 --n2 524288 --shapes 4:1,1:4,2:2 >> $O/diag0.txt 2>&1 || exit 4
timeout -k 10 240 python3 -u tools/rect_time.py --n1 524288 --n2 65536 --shapes 4:1,1:4,2:2 >> $O/diag0.txt 2>&1 || exit 5
echo done >> $O/diag0.txt
