# where the feeder's stalls are: per-strip feeder diagnostics in the horizontal band trace
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
F=$PWD/fast-needleman-wunsch_amd/build/libnwhip_frr.so
for v in a b; do
  NWHIP_LIB=$F timeout -k 10 150 python -u tools/tband_trace.py --n2 65536 > $O/tband_frr_$v.txt 2>&1 || exit 11
done
echo done > $O/done
