#!/bin/bash
# Instruction-cache counters over one timing-only fill (x22 experiment build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/icache; mkdir -p $OUT
export TMPDIR=/tmp; cd /tmp || exit 1
NWHIP_LIB=$R/fast-needleman-wunsch_amd/build/libnwhip_x22.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $OUT/p2 -o pmc -- python3 $R/tools/quick_time.py --sizes 262144 --reps 1 --flags 513 > $OUT/p2.log 2>&1
echo rc=$? >> $OUT/status.txt
