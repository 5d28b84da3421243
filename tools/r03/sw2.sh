#!/bin/bash
# SW traceback window geometry sweep (band half-width x windows per round)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03s
mkdir -p $O
cd $R
for b in 64 128; do for w in 128 256 512 4096; do
  NW_TB_BAND=$b NW_TB_MAXWIN=$w NW_TB_DEBUG=1 timeout -k 10 120 python3 -u bench.py --workload sw --steps 3 --warmup 1 > $O/g_${b}_${w}.json 2> $O/g_${b}_${w}.err || exit 1
  echo "band $b maxwin $w $(python3 -c "import json;d=json.load(open('$O/g_${b}_${w}.json'));print(d['traceback_ms_avg'], d['result_ok'])") $(tail -1 $O/g_${b}_${w}.err)" >> $O/geom.txt
done; done
