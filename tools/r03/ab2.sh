#!/bin/bash
# same-box A/B at 256k (4,4): r03a (chain1 row form) vs main (short-chain row form); then panel tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
B=$R/fast-needleman-wunsch_amd/build
for round in 1 2; do
  for v in r03a main; do
    lib=$B/libnwhip_$v.so; [ $v = main ] && lib=$B/libnwhip.so
    echo "== $v round $round" >> $O/ab2.txt
    NWHIP_LIB=$lib timeout -k 10 200 python3 -u tools/quick_time.py --sizes 262144 --kernel 2 --shapes 4:4 --reps 3 >> $O/ab2.txt 2>&1 || exit 3
  done
done
timeout -k 10 300 python3 -u tools/quick_time.py --sizes 65536,131072 --kernel 2 --shapes 4:1,2:2,1:4,2:4 --reps 2 >> $O/ab2.txt 2>&1 || exit 5
timeout -k 10 600 python3 -u -m pytest tests/test_panels.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/panels_tests5.txt 2>&1
echo "pytest rc=$?" >> $O/panels_tests5.txt
echo done >> $O/ab2.txt
