# compute wave cycles per step inside run_iter with and without the feeder (horizontal band)
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
F=$PWD/fast-needleman-wunsch_amd/build/libnwhip_frr.so
for v in def frr def2 frr2; do
  case $v in frr*) export NWHIP_LIB=$F;; *) unset NWHIP_LIB;; esac
  timeout -k 10 150 python -u tools/tband_trace.py --n2 65536 > $O/tband_$v.txt 2>&1 || exit 11
done
echo done > $O/done
