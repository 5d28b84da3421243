#!/bin/bash
# 2 ranks sharing one GPU (128 workers each) on half of config 4's per-GPU table: 2 bands of
# 32768 rows x 524288 columns, horizontal vs vertical sweep (real IPC feed / halo buffers)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03z
mkdir -p $O
cd $R
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29531 bench.py --gpus 2 --share-gpu --band-rows 32768 --band-sweep horizontal --alt-partition rows --steps 3 --warmup 1 --no-cpu-baseline > $O/share2_h.json 2> $O/share2_h.err || exit 1
