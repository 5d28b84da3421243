#!/bin/bash
# block-cyclic bands: parity, then 2- and 3-process shared-GPU bench rehearsals
# (every leg: cyclic rows, contiguous rows, columns), then the whole GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03c
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_cycles.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/cycles.txt 2>&1 || exit 1
for n in 2 3; do
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29517 \
   bench.py --gpus $n --share-gpu --band-rows 16384 --col-rows 131072 --col-width 65536 --steps 3 --warmup 1 --no-cpu-baseline > $O/share$n.json 2> $O/share$n.err || exit 2
done
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.txt 2>&1 || exit 3
