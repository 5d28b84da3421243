#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
true
for f in 0 1 8; do
  timeout -k 10 200 python3 -u tools/panel_trace.py --shape 4:4 --flags $f >> $O/panel_trace.txt 2>&1 || exit 3
done
timeout -k 10 200 python3 -u tools/panel_trace.py --shape 2:8 --flags 0 >> $O/panel_trace.txt 2>&1 || exit 4
echo done >> $O/panel_trace.txt
