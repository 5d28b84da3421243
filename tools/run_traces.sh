#!/bin/bash
# Strip-trace a set of fills on the GPU box.
# Usage: tools/run_traces.sh <outdir> <n> "<sub> <nc> <flags> [lib]" ...
set -o pipefail
O=gpurun_out/$1; N=$2; shift 2
mkdir -p $O
for cfg in "$@"; do
  set -- $cfg
  lib=${4:-}
  tag=$1_$2_$3${lib:+_$(basename $lib .so)}
  NWHIP_LIB=${lib:+$PWD/fast-needleman-wunsch_amd/build/$lib} timeout -k 10 200 \
      python3 tools/trace_strips.py --n $N --sub $1 --nc $2 --flags $3 > $O/tr_$tag.txt 2>&1 || exit 1
done
