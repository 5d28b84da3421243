#!/bin/bash
# chain2 (default build) tests + trace, chain1 variant trace (same box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_panels.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/panels_tests4.txt 2>&1
echo "pytest rc=$?" >> $O/panels_tests4.txt
for f in 0 8; do
  timeout -k 10 200 python3 -u tools/panel_trace.py --shape 4:4 --flags $f >> $O/panel_trace4.txt 2>&1 || exit 3
done
echo "--- chain1 variant" >> $O/panel_trace4.txt
for f in 0 8; do
  NWHIP_LIB=$R/fast-needleman-wunsch_amd/build/libnwhip_chain1.so timeout -k 10 200 python3 -u tools/panel_trace.py --shape 4:4 --flags $f >> $O/panel_trace4.txt 2>&1 || exit 4
done
timeout -k 10 300 python3 -u tools/quick_time.py --sizes 65536 --kernel 2 --shapes 4:1,2:2,1:4 --reps 2 >> $O/panel_trace4.txt 2>&1 || exit 5
echo done >> $O/panel_trace4.txt
