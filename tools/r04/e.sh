# Granule prefetch distance A/B (GPD=1 default vs GPD=3 = round 3), horizontal publish from
# the store waves: SW fill + hop, horizontal band hop, local 2-band sweeps, share-2 legs,
# vertical band trace, bench; then the GPU suite at the default
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
G3=$PWD/fast-needleman-wunsch_amd/build/libnwhip_gpd3.so
timeout -k 10 300 python -u -m pytest tests/test_sw.py tests/test_tbands.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/quicktest.txt 2>&1 || exit 10
for v in d3 d1; do
  if [ $v = d3 ]; then export NWHIP_LIB=$G3; else unset NWHIP_LIB; fi
  timeout -k 10 150 python -u tools/sw_shapes.py --shapes 2:2,4:1 > $O/sw_shapes_$v.txt 2>&1 || exit 11
  timeout -k 10 120 python -u tools/trace_strips.py --n 65536 --sw --sub 2 --nc 2 > $O/sw_trace_$v.txt 2>&1 || exit 12
  timeout -k 10 200 python -u tools/tband_trace.py --n2 65536 > $O/tband_$v.txt 2>&1 || exit 13
  timeout -k 10 150 python -u tools/local_tband_trace.py > $O/local_tband_$v.txt 2>&1 || exit 14
  timeout -k 10 150 python -u tools/local_bands_time.py > $O/local_$v.txt 2>&1 || exit 15
  timeout -k 10 200 python -u tools/vband_trace.py --waves 256,192 --save $O/vband_$v > $O/vband_$v.txt 2>&1 || exit 16
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 17
done
unset NWHIP_LIB
for sw in vertical horizontal; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29517 \
    bench.py --gpus 2 --steps 5 --warmup 2 --share-gpu --band-rows 32768 --band-sweep $sw --alt-partition none --no-cpu-baseline \
    > $O/share2_$sw.json 2> $O/share2_$sw.err || exit 18
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gputest.txt 2>&1 || exit 19
echo done > $O/done
