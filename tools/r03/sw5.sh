#!/bin/bash
# SW fill with the 3-VALU cell: SW tests, strip shapes at 64k, bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03w
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_sw.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/sw_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/sw_shapes.py --shapes 4:1,2:2,2:1,1:4 > $O/sw_shapes.txt 2>&1 || exit 2
timeout -k 10 300 python3 -u bench.py --workload sw --steps 10 --warmup 2 > $O/sw_bench.json 2> $O/sw_bench.err || exit 3
