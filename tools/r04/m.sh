# wave -> SIMD placement probe; compute roles on the waves alone on their SIMD (rr) vs identity
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
RR=$PWD/fast-needleman-wunsch_amd/build/libnwhip_rr.so
timeout -k 10 60 tools/ubench/wave_simd > $O/wave_simd.txt 2>&1 || exit 9
NWHIP_LIB=$RR timeout -k 10 300 python -u -m pytest tests/test_sw.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/test_rr.txt 2>&1 || exit 10
for v in def rr def2 rr2; do
  case $v in rr*) export NWHIP_LIB=$RR;; *) unset NWHIP_LIB;; esac
  timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2,1:4 --reps 3 > $O/sw_shapes_$v.txt 2>&1 || exit 11
done
for v in def rr; do
  case $v in rr*) export NWHIP_LIB=$RR;; *) unset NWHIP_LIB;; esac
  timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 > $O/sw_trace_$v.txt 2>&1 || exit 12
  timeout -k 10 200 python -u tools/vband_trace.py --waves 256 --save $O/vband_$v > $O/vband_$v.txt 2>&1 || exit 13
  timeout -k 10 150 python -u tools/rect_time.py --n1 524288 --n2 65536 --shapes 2:2,1:4 --kernel 1 > $O/rect_$v.txt 2>&1 || exit 14
done
echo done > $O/done
