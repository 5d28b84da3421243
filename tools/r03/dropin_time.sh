#!/bin/bash
# drop-in CLI timings (driver.cpp's own timer) on the 8gb and big fixtures next to
# the bare D2H of the same table (tools/d2h_bench), on the GPU box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
G=tests/golden/bdna
for name in 8gb big; do
  if [ $name = big ]; then a=$G/big1.bdna; b=$G/big2.bdna; else a=$G/$name-1.bdna; b=$G/$name-2.bdna; fi
  for exe in oracle/_ref/ref_driver_hip fast-needleman-wunsch_amd/build/nw_driver; do
    for mode in warm cold; do
      for rep in 1 2; do
        echo "== $name $exe $mode rep $rep" >> $O/dropin_time.txt
        cs=""; [ $mode = cold ] && cs=1
        t0=$(date +%s.%N); NW_COLD_START=$cs NW_HOST_TIMING=1 timeout -k 10 300 $exe $a $b >> $O/dropin_time.txt 2>&1 || exit 3; t1=$(date +%s.%N); python3 -c "print('wall %.3f s' % ($t1 - $t0))" >> $O/dropin_time.txt
      done
    done
  done
done
true
echo done >> $O/dropin_time.txt
