# idle-feeder poll period A/B: s32 / s127 = NW_FEEDER + NW_ROLE_RR + s_sleep(32 / 127) between
# empty polls, vs default; horizontal band
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
B=$PWD/fast-needleman-wunsch_amd/build
NWHIP_LIB=$B/libnwhip_s127.so timeout -k 10 300 python -u -m pytest tests/test_tbands.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/test_s127.txt 2>&1 || exit 10
for v in def s32 s127 def2 s32b s127b; do
  case $v in s32*) export NWHIP_LIB=$B/libnwhip_s32.so;; s127*) export NWHIP_LIB=$B/libnwhip_s127.so;; *) unset NWHIP_LIB;; esac
  timeout -k 10 150 python -u tools/tband_trace.py --n2 65536 > $O/tband_$v.txt 2>&1 || exit 11
done
echo done > $O/done
