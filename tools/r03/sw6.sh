#!/bin/bash
# config 5 at the round-end kernel: bench line + rocprofv3 kernel stats of the same command
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03f
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --workload sw --steps 10 --warmup 2 > $O/sw_bench2.json 2> $O/sw_bench2.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/swkt -o kt -- python3 $R/bench.py --workload sw --steps 10 --warmup 2 > $O/swkt.log 2>&1 || exit 2
