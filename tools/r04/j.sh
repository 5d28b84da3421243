# non-temporal table stores in the horizontal strips (trnt) vs default: band alone + trace
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
NT=$PWD/fast-needleman-wunsch_amd/build/libnwhip_trnt.so
for v in def nt def2 nt2; do
  case $v in nt*) export NWHIP_LIB=$NT;; *) unset NWHIP_LIB;; esac
  timeout -k 10 150 python -u tools/band_alone.py --rank 7 --sweep horizontal --reps 4 > $O/alone_$v.txt 2>&1 || exit 11
  timeout -k 10 150 python -u tools/tband_trace.py --n2 65536 > $O/tband_$v.txt 2>&1 || exit 12
done
unset NWHIP_LIB
NWHIP_LIB=$NT timeout -k 10 300 python -u -m pytest tests/test_tbands.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tbtest_nt.txt 2>&1 || exit 13
echo done > $O/done
