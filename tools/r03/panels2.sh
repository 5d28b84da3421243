#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_panels.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/panels_tests2.txt 2>&1
echo "pytest rc=$?" >> $O/panels_tests2.txt
for sh in 4:4 2:4; do
  timeout -k 10 200 python3 -u tools/panel_trace.py --shape $sh --flags 0 >> $O/panel_trace2.txt 2>&1 || exit 3
done
timeout -k 10 200 python3 -u tools/panel_trace.py --shape 4:4 --flags 8 >> $O/panel_trace2.txt 2>&1 || exit 4
echo done >> $O/panel_trace2.txt
