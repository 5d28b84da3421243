#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03c
mkdir -p $O
cd $R
echo "GPU_MAX_HW_QUEUES=$GPU_MAX_HW_QUEUES" > $O/loop.txt
timeout -k 10 120 python3 -u tools/r03/cyc_loop.py 3 2 1000 64 >> $O/loop.txt 2>&1 || exit 1
timeout -k 10 120 python3 -u tools/r03/cyc_loop.py 3 2 1000 64 16 >> $O/loop.txt 2>&1 || exit 2
timeout -k 10 120 python3 -u tools/r03/cyc_loop.py 2 4 1000 64 >> $O/loop.txt 2>&1 || exit 3
