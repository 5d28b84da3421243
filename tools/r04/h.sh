# granule prefetch distance 2 for the C = 2 shapes (gpd2) vs the default 3: SW fill + trace,
# vertical band; the compute-wave iteration in isolation (step_loop, NW and SW)
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
G2=$PWD/fast-needleman-wunsch_amd/build/libnwhip_gpd2.so
timeout -k 10 120 tools/ubench/step_loop > $O/step_loop.txt 2>&1 || exit 9
NWHIP_LIB=$G2 timeout -k 10 300 python -u -m pytest tests/test_sw.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/swtest_gpd2.txt 2>&1 || exit 10
for v in def gpd2 def2 gpd22; do
  case $v in gpd2*) export NWHIP_LIB=$G2;; *) unset NWHIP_LIB;; esac
  timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2 --reps 5 > $O/sw_shapes_$v.txt 2>&1 || exit 11
done
for v in def gpd2; do
  case $v in gpd2*) export NWHIP_LIB=$G2;; *) unset NWHIP_LIB;; esac
  timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 > $O/sw_trace_$v.txt 2>&1 || exit 12
  timeout -k 10 200 python -u tools/vband_trace.py --waves 256 --save $O/vband_$v > $O/vband_$v.txt 2>&1 || exit 13
done
echo done > $O/done
