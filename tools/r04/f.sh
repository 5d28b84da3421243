# compute-wave priority (NW_COMPUTE_PRIO=2) and 3 store waves per C=2 ring (NW_SPR2=3) A/B
# against the default, local horizontal timing discrepancy (wall vs events, traced vs
# untraced), then the GPU suite
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
B=$PWD/fast-needleman-wunsch_amd/build
timeout -k 10 300 python -u -m pytest tests/test_sw.py tests/test_tbands.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/quicktest.txt 2>&1 || exit 10
for v in def prio spr3 def2; do
  case $v in prio) export NWHIP_LIB=$B/libnwhip_prio.so;; spr3) export NWHIP_LIB=$B/libnwhip_spr3.so;; *) unset NWHIP_LIB;; esac
  timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2,4:1 > $O/sw_shapes_$v.txt 2>&1 || exit 11
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 12
  if [ $v != def2 ]; then
    timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 > $O/sw_trace_$v.txt 2>&1 || exit 13
    timeout -k 10 200 python -u tools/vband_trace.py --waves 256 --save $O/vband_$v > $O/vband_$v.txt 2>&1 || exit 15
  fi
done
unset NWHIP_LIB
timeout -k 10 200 python -u tools/tband_trace.py --n2 65536 > $O/tband.txt 2>&1 || exit 14
timeout -k 10 150 python -u tools/local_tband_trace.py > $O/local_tband.txt 2>&1 || exit 16
timeout -k 10 150 python -u tools/local_bands_time.py --only horizontal > $O/local_h.txt 2>&1 || exit 17
timeout -k 10 150 python -u tools/local_bands_time.py > $O/local_both.txt 2>&1 || exit 18
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gputest.txt 2>&1 || exit 19
echo done > $O/done
