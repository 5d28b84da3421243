# panel kernel: left values loaded after a group's second row (NW_ROWS_MIDFEED, lead 6
# rows) vs before the group (default, lead 8): parity, interleaved A/B at 256k, trace
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
B=$PWD/fast-needleman-wunsch_amd/build
NWHIP_LIB=$B/libnwhip_mid.so timeout -k 10 400 python3 -u -m pytest tests/test_panels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_mid.txt 2>&1 || exit 1
for i in 1 2 3; do
  for v in "" _mid; do
    echo "lib$v" >> $O/pan_ab.txt
    NWHIP_LIB=$B/libnwhip$v.so timeout -k 10 300 python3 -u tools/quick_time.py --sizes 262144 --kernel 2 --reps 4 >> $O/pan_ab.txt 2>&1 || exit 2
  done
done
for v in "" _mid; do
  NWHIP_LIB=$B/libnwhip$v.so timeout -k 10 300 python3 -u tools/panel_trace.py > $O/pan_trace$v.txt 2>&1 || exit 3
done
echo done > $O/done
