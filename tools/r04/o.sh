# feeder wave + compute role alone on its SIMD, the feeder reading the error word every 32
# empty polls (frr) vs default: horizontal band, SW fill
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
F=$PWD/fast-needleman-wunsch_amd/build/libnwhip_frr.so
NWHIP_LIB=$F timeout -k 10 300 python -u -m pytest tests/test_tbands.py tests/test_sw.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/test_frr.txt 2>&1 || exit 10
for v in def frr def2 frr2; do
  case $v in frr*) export NWHIP_LIB=$F;; *) unset NWHIP_LIB;; esac
  timeout -k 10 150 python -u tools/tband_trace.py --n2 65536 > $O/tband_$v.txt 2>&1 || exit 11
  timeout -k 10 150 python -u tools/local_tband_trace.py --plain-reps 2 > $O/local_$v.txt 2>&1 || exit 13
  timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2 --reps 3 > $O/sw_$v.txt 2>&1 || exit 14
done
echo done > $O/done
