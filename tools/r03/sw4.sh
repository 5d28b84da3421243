#!/bin/bash
# config 5 at the new traceback defaults: SW tests, bench lines (both schemes), kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03t
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_sw.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/sw_tests.txt 2>&1 || exit 1
NW_TB_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload sw --steps 10 --warmup 2 > $O/sw_bench.json 2> $O/sw_bench.err || exit 2
NW_TB_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload sw --scheme 1,0,-1 --steps 10 --warmup 2 > $O/sw_bench_shipped.json 2> $O/sw_bench_shipped.err || exit 3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/bench.py --workload sw --steps 5 --warmup 2 > $O/kt.log 2>&1 || exit 4
