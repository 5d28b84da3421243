#!/bin/bash
# SQ counters of the solo-strip timing (tools/solo_strip.py) for one library build.
# Usage: tools/pmc_solo.sh <outdir> <lib suffix ("" = default)> <C>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; V=$2; C=${3:-2}
mkdir -p $OUT
export TMPDIR=/tmp
export NWHIP_LIB=$R/fast-needleman-wunsch_amd/build/libnwhip$V.so
cd /tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o pmc -- python3 $R/tools/solo_strip.py --sub $C > $OUT/pmc$i.log 2>&1 || { echo "pass $i failed rc=$?" >> $OUT/status.txt; exit 1; }
done
echo done >> $OUT/status.txt
