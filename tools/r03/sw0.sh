#!/bin/bash
# SW config 5: fill time per kernel family / shape, then the bench line and a kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03s
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/sw_shapes.py > $O/sw_shapes.txt 2>&1 || exit 1
NW_TB_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload sw --steps 5 --warmup 2 > $O/sw_bench.json 2> $O/sw_bench.err || exit 2
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/bench.py --workload sw --steps 5 --warmup 2 > $O/kt.log 2>&1 || exit 3
