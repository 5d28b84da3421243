# panel kernel: left values loaded after the group (late feed) only in the first / last
# trips of a panel (NW_ROWS_LATE_HEAD / _TAIL) vs always before (default) / always after:
# parity of the head+tail variant, interleaved A/B at 256k, panel traces
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
B=$PWD/fast-needleman-wunsch_amd/build
NWHIP_LIB=$B/libnwhip_lh2t2.so timeout -k 10 400 python3 -u -m pytest tests/test_panels.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/panels_lh2t2_tests.txt 2>&1 || exit 1
for i in 1 2; do
  for v in "" _lh1 _lh4 _lt1 _lh2t2 _late; do
    echo "lib$v" >> $O/pan_ab.txt
    NWHIP_LIB=$B/libnwhip$v.so timeout -k 10 300 python3 -u tools/quick_time.py --sizes 262144 --kernel 2 --reps 4 >> $O/pan_ab.txt 2>&1 || exit 2
  done
done
for v in "" _lh4 _lh2t2; do
  NWHIP_LIB=$B/libnwhip$v.so timeout -k 10 300 python3 -u tools/panel_trace.py > $O/pan_trace$v.txt 2>&1 || exit 3
done
echo done > $O/done
