# A/B pipelined vs serial polls on one box (bench line incl. config5), band alone, SW probe
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
SER=$PWD/fast-needleman-wunsch_amd/build/libnwhip_serialpoll.so
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_pipe$i.json 2> $O/bench_pipe$i.err || exit 11
  NWHIP_LIB=$SER timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_serial$i.json 2> $O/bench_serial$i.err || exit 12
done
for r in 0 7; do for s in vertical horizontal; do timeout -k 10 120 python -u tools/band_alone.py --rank $r --sweep $s >> $O/alone.txt 2>&1 || exit 16; done; done
timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2,4:1,1:4,2:1 > $O/sw_shapes.txt 2>&1 || exit 21
timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2,4:1,1:4,2:1 --flags 1 >> $O/sw_shapes.txt 2>&1 || exit 22
NWHIP_LIB=$SER timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2,4:1 > $O/sw_shapes_serial.txt 2>&1 || exit 23
timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 > $O/sw_trace.txt 2>&1 || exit 24
timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 --flags 1 > $O/sw_trace_nostore.txt 2>&1 || exit 25
echo done > $O/done
