#!/bin/bash
# horizontal-strip row bands: config-4 geometry every row, shared-GPU 2-process bench legs,
# a 2-rank shared-GPU bench at the config-4 band width
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03h
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_full_size.py tests/test_bands.py -m gpu -x -v -k "config4_band_geometry or two_process_bands" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tbands2.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tbands2.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29517 bench.py --gpus 2 --share-gpu --band-rows 16384 --steps 5 --warmup 2 --no-cpu-baseline > $O/share2.json 2> $O/share2.err || exit 41
