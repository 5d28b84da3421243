#!/bin/bash
# per-GPU column-band geometry (65536 cols x 524288 rows): paces of strips and panels,
# with stores and compute-only (flags 8); then the SW window-geometry sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03r
mkdir -p $O
cd $R
for k in 1 2; do for f in 0 8; do
  timeout -k 10 200 python3 -u tools/rect_time.py --n1 65536 --n2 524288 --kernel $k --flags $f --shapes 4:1,2:2,1:4 --reps 2 >> $O/rect.txt 2>&1 || exit 1
done; done
timeout -k 10 200 python3 -u tools/rect_time.py --n1 524288 --n2 65536 --kernel 2 --shapes 4:4,4:1,1:4 --reps 2 >> $O/rect.txt 2>&1 || exit 2
bash tools/r03/sw2.sh
