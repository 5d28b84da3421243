# Round-4 GPU pass: the GPU suite, the default bench line, then measurements
# (config-4 band traversal vs resident strips, 2 local bands both sweeps, pipelined
# vs serial polls, one rank's band alone, SW fill probe)
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
SER=$PWD/fast-needleman-wunsch_amd/build/libnwhip_serialpoll.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gputest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gputest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 11; fi
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 12
timeout -k 10 300 python -u tools/vband_trace.py > $O/vband.txt 2>&1 || exit 13
timeout -k 10 150 python -u tools/local_bands_time.py > $O/local.txt 2>&1 || exit 14
NWHIP_LIB=$SER timeout -k 10 150 python -u tools/local_bands_time.py > $O/local_serial.txt 2>&1 || exit 15
for r in 0 7; do for s in vertical horizontal; do timeout -k 10 120 python -u tools/band_alone.py --rank $r --sweep $s >> $O/alone.txt 2>&1 || exit 16; done; done
timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2,4:1,1:4,2:1 > $O/sw_shapes.txt 2>&1 || exit 21
timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2,4:1,1:4,2:1 --flags 1 >> $O/sw_shapes.txt 2>&1 || exit 22
NWHIP_LIB=$SER timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2,4:1 > $O/sw_shapes_serial.txt 2>&1 || exit 23
timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 > $O/sw_trace.txt 2>&1 || exit 24
timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 --flags 1 > $O/sw_trace_nostore.txt 2>&1 || exit 25
echo done > $O/done
