set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_bands.py tests/test_tbands.py > $O/r04g_bands.txt 2>&1 || exit 11
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/r04g_bench.json 2> $O/r04g_bench.err || exit 12
NWHIP_LIB=$PWD/fast-needleman-wunsch_amd/build/libnwhip_serialpoll.so timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/r04g_bench_serial.json 2> $O/r04g_bench_serial.err || exit 13
timeout -k 10 120 python -u tools/local_bands_time.py > $O/r04g_local.txt 2>&1 || exit 14
NWHIP_LIB=$PWD/fast-needleman-wunsch_amd/build/libnwhip_serialpoll.so timeout -k 10 120 python -u tools/local_bands_time.py > $O/r04g_local_serial.txt 2>&1 || exit 15
for r in 0 3 7; do for s in vertical horizontal; do timeout -k 10 100 python -u tools/band_alone.py --rank $r --sweep $s >> $O/r04g_alone.txt 2>&1 || exit 16; done; done
# SW config-5 fill probe: shapes with and without table stores, per-strip trace, poll A/B
set -o pipefail
O=gpurun_out
SER=$PWD/fast-needleman-wunsch_amd/build/libnwhip_serialpoll.so
timeout -k 10 120 python -u tools/sw_shapes.py --shapes 2:2,4:1,1:4,2:1 > $O/r04h_sw_shapes.txt 2>&1 || exit 21
timeout -k 10 120 python -u tools/sw_shapes.py --shapes 2:2,4:1,1:4,2:1 --flags 1 >> $O/r04h_sw_shapes.txt 2>&1 || exit 22
NWHIP_LIB=$SER timeout -k 10 120 python -u tools/sw_shapes.py --shapes 2:2,4:1 > $O/r04h_sw_shapes_serial.txt 2>&1 || exit 23
timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 > $O/r04h_sw_trace.txt 2>&1 || exit 24
NWHIP_LIB=$SER timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 > $O/r04h_sw_trace_serial.txt 2>&1 || exit 25
