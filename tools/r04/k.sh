# Round-4 final state on a fresh box: smoke, the GPU suite, the driver's default bench line,
# and the drop-in CLI on `big` cold (default) and warm (NW_WARM_START=1)
set -o pipefail
O=gpurun_out/r04z
mkdir -p $O
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 10
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gputest.txt 2>&1 || exit 11
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 12
G=tests/golden/bdna
for mode in cold warm; do
  for rep in 1 2; do
    echo "== big nw_driver $mode rep $rep" >> $O/dropin.txt
    if [ $mode = warm ]; then export NW_WARM_START=1; else unset NW_WARM_START; fi
    NW_HOST_TIMING=1 timeout -k 10 120 fast-needleman-wunsch_amd/build/nw_driver $G/big1.bdna $G/big2.bdna >> $O/dropin.txt 2>&1 || exit 13
  done
done
echo done > $O/done
