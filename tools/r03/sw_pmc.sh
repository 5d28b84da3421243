#!/bin/bash
# config 5 (SW 64k): kernel stats + WRITE_SIZE / FETCH_SIZE passes per kernel; the
# block-cyclic decomposition cost on one GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03p
mkdir -p $O
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 python3 $R/bench.py --workload sw --steps 5 --warmup 2 > $O/sw_bench.json 2> $O/sw_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/bench.py --workload sw --steps 5 --warmup 2 > $O/kt.log 2>&1 || exit 2
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o pmc -- python3 $R/bench.py --workload sw --steps 3 --warmup 1 > $O/pmc_w.log 2>&1 || exit 3
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o pmc -- python3 $R/bench.py --workload sw --steps 3 --warmup 1 > $O/pmc_f.log 2>&1 || exit 4
cd $R
timeout -k 10 300 python3 -u tools/cycle_time.py > $O/cycle_time.txt 2>&1 || exit 5
