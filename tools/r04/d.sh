# SW strip cell in the w form + serial polls: SW tests first, the GPU suite, bench, SW trace
set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sw.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/swtest.txt 2>&1 || exit 10
timeout -k 10 200 python -u tools/sw_shapes.py --shapes 2:2,4:1,1:4,2:1 > $O/sw_shapes.txt 2>&1 || exit 11
timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 > $O/sw_trace.txt 2>&1 || exit 12
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 13
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gputest.txt 2>&1 || exit 14
timeout -k 10 300 python -u tools/vband_trace.py --waves 256,192 --save $O/vband > $O/vband.txt 2>&1 || exit 15
timeout -k 10 200 python -u tools/tband_trace.py --n2 65536 > $O/tband.txt 2>&1 || exit 16
timeout -k 10 120 tools/ubench/tile_step > $O/tile_step.txt 2>&1 || exit 17
timeout -k 10 120 tools/ubench/cu_store > $O/cu_store.txt 2>&1 || exit 18
timeout -k 10 150 python -u tools/local_tband_trace.py > $O/local_tband.txt 2>&1 || exit 19
NW_LINK_COARSE=1 timeout -k 10 150 python -u tools/local_tband_trace.py > $O/local_tband_coarse.txt 2>&1 || exit 20
echo done > $O/done
