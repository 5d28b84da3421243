# (4,1) feeder wave with the compute role on a SIMD of its own (frr: NW_FEEDER + NW_ROLE_RR)
# vs default, for the horizontal band (the N > 1 value's sweep)
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
F=$PWD/fast-needleman-wunsch_amd/build/libnwhip_frr.so
NWHIP_LIB=$F timeout -k 10 300 python -u -m pytest tests/test_tbands.py tests/test_config4.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/test_frr.txt 2>&1 || exit 10
for v in def frr def2 frr2; do
  case $v in frr*) export NWHIP_LIB=$F;; *) unset NWHIP_LIB;; esac
  timeout -k 10 150 python -u tools/tband_trace.py --n2 65536 > $O/tband_$v.txt 2>&1 || exit 11
  timeout -k 10 150 python -u tools/band_alone.py --rank 7 --sweep horizontal --reps 3 > $O/alone_$v.txt 2>&1 || exit 12
  timeout -k 10 150 python -u tools/local_tband_trace.py --plain-reps 2 > $O/local_$v.txt 2>&1 || exit 13
done
echo done > $O/done
