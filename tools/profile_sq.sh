#!/bin/bash
# SQ / LDS counter passes (rocprofv3 --pmc, one pass per counter set, each its own
# run) over one fill of size N: attributes where the strip kernel's wave time goes.
# Usage: tools/profile_sq.sh <outdir> <n> [extra quick_time args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; N=${2:-131072}; shift 2
EXTRA="$@"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc$i" -o pmc -- \
      python3 "$R/tools/quick_time.py" --sizes "$N" --reps 1 $EXTRA > "$OUT/pmc$i.log" 2>&1 || { echo "pass $i rc=$?" >> "$OUT/status.txt"; exit 20; }
done
echo done >> "$OUT/status.txt"
