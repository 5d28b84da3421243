#!/bin/bash
# panel kernel A/B: row characters by s_load (shipped) vs vector load (NW_ROWS_VLOAD)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03u
mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 300 python3 -u tools/quick_time.py --sizes 262144 --kernel 2 --reps 5 >> $O/pan_ab.txt 2>&1 || exit 31
  NWHIP_LIB=$R/fast-needleman-wunsch_amd/build/libnwhip_vload.so timeout -k 10 300 python3 -u tools/quick_time.py --sizes 262144 --kernel 2 --reps 5 >> $O/pan_ab.txt 2>&1 || exit 32
done
