# Round-4 final state on a fresh box: smoke, the GPU suite, the driver's default bench line,
# and the drop-in CLI on `big` cold (default) and warm (NW_WARM_START=1)
set -o pipefail
O=gpurun_out/r04z2
mkdir -p $O
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 10
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gputest.txt 2>&1 || exit 11
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 12
echo done > $O/done
