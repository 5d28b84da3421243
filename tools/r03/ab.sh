#!/bin/bash
# same-box A/B of panel-kernel builds at 256k (4,4): r03a (committed 47 ms kernel), chain1, chain2 (default)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
B=$R/fast-needleman-wunsch_amd/build
for round in 1 2; do
  for v in r03a chain1 main; do
    lib=$B/libnwhip_$v.so; [ $v = main ] && lib=$B/libnwhip.so
    echo "== $v round $round" >> $O/ab.txt
    NWHIP_LIB=$lib timeout -k 10 200 python3 -u tools/quick_time.py --sizes 262144 --kernel 2 --shapes 4:4 --reps 3 >> $O/ab.txt 2>&1 || exit 3
  done
done
echo done >> $O/ab.txt
