set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_bands.py tests/test_tbands.py > $O/r04g_bands.txt 2>&1 || exit 11
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/r04g_bench.json 2> $O/r04g_bench.err || exit 12
NWHIP_LIB=$PWD/fast-needleman-wunsch_amd/build/libnwhip_serialpoll.so timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/r04g_bench_serial.json 2> $O/r04g_bench_serial.err || exit 13
timeout -k 10 120 python -u tools/local_bands_time.py > $O/r04g_local.txt 2>&1 || exit 14
NWHIP_LIB=$PWD/fast-needleman-wunsch_amd/build/libnwhip_serialpoll.so timeout -k 10 120 python -u tools/local_bands_time.py > $O/r04g_local_serial.txt 2>&1 || exit 15
for r in 0 3 7; do for s in vertical horizontal; do timeout -k 10 100 python -u tools/band_alone.py --rank $r --sweep $s >> $O/r04g_alone.txt 2>&1 || exit 16; done; done
