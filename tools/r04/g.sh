# strip feeder wave (default) vs none (NW_NO_FEEDER): parity first, then SW fill + hop,
# horizontal band hop, local 2 bands, vertical band trace, bench; GPU suite at the end
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
NF=$PWD/fast-needleman-wunsch_amd/build/libnwhip_nofeed.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_sw.py tests/test_tbands.py tests/test_bands.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/quicktest.txt 2>&1 || exit 10
for v in feed nofeed; do
  if [ $v = nofeed ]; then export NWHIP_LIB=$NF; else unset NWHIP_LIB; fi
  timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2,4:1 > $O/sw_shapes_$v.txt 2>&1 || exit 11
  timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 > $O/sw_trace_$v.txt 2>&1 || exit 12
  timeout -k 10 200 python -u tools/tband_trace.py --n2 65536 > $O/tband_$v.txt 2>&1 || exit 13
  timeout -k 10 150 python -u tools/local_tband_trace.py --plain-reps 2 > $O/local_tband_$v.txt 2>&1 || exit 14
  timeout -k 10 200 python -u tools/vband_trace.py --waves 256 --save $O/vband_$v > $O/vband_$v.txt 2>&1 || exit 15
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 16
done
unset NWHIP_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gputest.txt 2>&1 || exit 19
echo done > $O/done
