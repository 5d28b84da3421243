#!/bin/bash
# SQ counter attribution of the horizontal band alone (one GPU's config-4 band geometry,
# 524288 x 65536, nw_fill_tband_async): separate rocprofv3 --pmc passes (<= 8 SQ
# counters each), for the normal fill and for the compute-only probe (flags 0x201:
# timing only + no store waves), so the store waves' share can be told apart.
# Usage: tools/profile_sq_band.sh <outdir>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
i=0
for flags in 0 513; do
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/f${flags}_p$i" -o pmc -- \
        python3 "$R/tools/tband_time.py" --reps 1 --vertical "" --flags $flags > "$OUT/f${flags}_p$i.log" 2>&1 \
        || { echo "pass $i (flags $flags) rc=$?" >> "$OUT/status.txt"; exit 20; }
  done
done
echo done >> "$OUT/status.txt"
