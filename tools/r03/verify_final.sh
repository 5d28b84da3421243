#!/bin/bash
# HEAD verification: full GPU suite + smoke, the default bench line, the SW bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03z
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gputest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 21
timeout -k 10 300 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit 22
timeout -k 10 300 python3 -u bench.py --workload sw --steps 10 --warmup 2 > $O/sw_bench.json 2> $O/sw_bench.err || exit 23
echo done > $O/done
