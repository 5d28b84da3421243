# Round-4 first GPU pass at HEAD: smoke, the whole GPU suite, the default bench line
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 10
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gputest.txt 2>&1 || exit 11
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 12
echo done > $O/done
