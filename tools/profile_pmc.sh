#!/bin/bash
# Collect rocprofv3 kernel-trace stats and PMC counters (separate passes) for one
# fill size.  Usage: tools/profile_pmc.sh <outdir> <n> [waves]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; N=${2:-131072}; W=${3:-0}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
APP="python3 $R/tools/quick_time.py --sizes $N --waves $W --reps 1"
timeout -k 10 240 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $APP > $OUT/kt.log 2>&1 || exit 1
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_MISC" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o pmc -- $APP > $OUT/pmc$i.log 2>&1 || echo "pass $i failed rc=$?" >> $OUT/status.txt
done
echo done >> $OUT/status.txt
