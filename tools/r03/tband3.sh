#!/bin/bash
# horizontal strips: where the per-column pace goes (stores to scratch, ring drained unread,
# no store waves), and the band time against its strip count (the hop)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03h
mkdir -p $O
cd $R
for f in 0 1 4 8; do
  timeout -k 10 200 python3 -u tools/tband_time.py --flags $f --vertical "" >> $O/tband_flags.txt 2>&1 || exit 31
done
for n2 in 256 512 1024 4096 16384; do
  timeout -k 10 200 python3 -u tools/tband_time.py --n2 $n2 --vertical "" --reps 5 >> $O/tband_hops.txt 2>&1 || exit 32
done
