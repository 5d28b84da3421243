#!/bin/bash
# SW traceback window geometry sweep with bands up to 256 (test first)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03s
mkdir -p $O
cd $R
NW_TB_BAND=256 timeout -k 10 300 python3 -u -m pytest tests/test_sw.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/sw_tests256.txt 2>&1 || exit 1
rm -f $O/geom2.txt
for b in 128 192 256; do for w in 128 256 512; do
  NW_TB_BAND=$b NW_TB_MAXWIN=$w NW_TB_DEBUG=1 timeout -k 10 120 python3 -u bench.py --workload sw --steps 3 --warmup 1 > $O/g_${b}_${w}.json 2> $O/g_${b}_${w}.err || exit 2
  NW_TB_BAND=$b NW_TB_MAXWIN=$w NW_TB_DEBUG=1 timeout -k 10 120 python3 -u bench.py --workload sw --scheme 1,0,-1 --steps 3 --warmup 1 > $O/h_${b}_${w}.json 2> $O/h_${b}_${w}.err || exit 3
  echo "band $b maxwin $w mm1 $(python3 -c "import json;d=json.load(open('$O/g_${b}_${w}.json'));print(d['traceback_ms_avg'], d['result_ok'])") $(tail -1 $O/g_${b}_${w}.err) | shipped $(python3 -c "import json;d=json.load(open('$O/h_${b}_${w}.json'));print(d['traceback_ms_avg'], d['result_ok'])") $(tail -1 $O/h_${b}_${w}.err)" >> $O/geom2.txt
done; done
