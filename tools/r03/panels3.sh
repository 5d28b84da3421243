#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
for f in 1 0; do
  timeout -k 10 200 python3 -u tools/panel_trace.py --shape 4:4 --flags $f >> $O/panel_trace3.txt 2>&1 || exit 3
done
timeout -k 10 300 python3 -u tools/quick_time.py --sizes 65536,32768 --kernel 2 --shapes 4:1,2:2,1:4 --reps 2 >> $O/panel_trace3.txt 2>&1 || exit 4
echo done >> $O/panel_trace3.txt
