# rebuilt library (version string only): smoke, the parity files, bench as the driver runs it
set -o pipefail
O=gpurun_out/r04z4
mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_panels.py tests/test_sw.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || exit 2
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit 3
echo done > $O/done
