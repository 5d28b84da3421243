# Rehearsal of the N > 1 bench's default path (horizontal row bands as value + the alternate
# legs) with 4 and 8 ranks sharing one GPU through IPC-mapped buffers
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
for n in 4 8; do
  br=$((65536 / n))
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr=127.0.0.1 --master-port=$((29600 + n)) \
    bench.py --gpus $n --steps 3 --warmup 2 --share-gpu --band-rows $br --col-width $br --col-rows 65536 --no-cpu-baseline \
    > $O/share${n}.json 2> $O/share${n}.err || exit 1$n
done
echo done > $O/done
