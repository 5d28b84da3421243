# SW config-5 fill probe: shapes with and without table stores, per-strip trace, poll A/B
set -o pipefail
O=gpurun_out
SER=$PWD/fast-needleman-wunsch_amd/build/libnwhip_serialpoll.so
timeout -k 10 120 python -u tools/sw_shapes.py --shapes 2:2,4:1,1:4,2:1 > $O/r04h_sw_shapes.txt 2>&1 || exit 21
timeout -k 10 120 python -u tools/sw_shapes.py --shapes 2:2,4:1,1:4,2:1 --flags 1 >> $O/r04h_sw_shapes.txt 2>&1 || exit 22
NWHIP_LIB=$SER timeout -k 10 120 python -u tools/sw_shapes.py --shapes 2:2,4:1 > $O/r04h_sw_shapes_serial.txt 2>&1 || exit 23
timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 > $O/r04h_sw_trace.txt 2>&1 || exit 24
NWHIP_LIB=$SER timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 > $O/r04h_sw_trace_serial.txt 2>&1 || exit 25
