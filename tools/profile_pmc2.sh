#!/bin/bash
# PMC passes for one fill config.  Usage: tools/profile_pmc2.sh <outdir> <n> <waves> <sub> <flags>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; N=$2; W=$3; K=$4; F=$5
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
APP="python3 $R/tools/quick_time.py --sizes $N --waves $W --sub $K --flags $F --reps 1"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL" \
           "SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_VMEM_WR SQ_INST_LEVEL_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o pmc -- $APP > $OUT/pmc$i.log 2>&1 || echo "pass $i failed rc=$?" >> $OUT/status.txt
done
echo done >> $OUT/status.txt
