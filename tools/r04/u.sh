# agent-scope granules (intra-GPU hand-offs; build NW_EXP_GRAN_AGENT) vs system scope: bench
# (256k panels + SW), horizontal and vertical band alone, SW fill; parity of the variant first
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
AG=$PWD/fast-needleman-wunsch_amd/build/libnwhip_ag.so
NWHIP_LIB=$AG timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_sw.py tests/test_tbands.py tests/test_panels.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/test_ag.txt 2>&1 || exit 10
for v in def ag def2 ag2; do
  case $v in ag*) export NWHIP_LIB=$AG;; *) unset NWHIP_LIB;; esac
  timeout -k 10 150 python -u tools/tband_trace.py --n2 65536 > $O/tband_$v.txt 2>&1 || exit 11
  timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2 --reps 3 > $O/sw_$v.txt 2>&1 || exit 12
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 13
done
echo done > $O/done
