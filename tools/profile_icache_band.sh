#!/bin/bash
# Instruction-cache and vector-memory issue counters of the horizontal band alone
# (524288 x 65536, tools/tband_time.py), separate rocprofv3 --pmc passes (2 SQC / <= 8 SQ
# counters each), KILL after 120 s per pass.  Usage: tools/profile_icache_band.sh <outdir>
# (NWHIP_LIB in the environment selects a library variant)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
i=0
for set in "SQC_ICACHE_REQ SQC_ICACHE_MISSES" "SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE" \
           "SQ_IFETCH SQ_INSTS_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o pmc -- \
      python3 "$R/tools/tband_time.py" --reps 1 --vertical "" > "$OUT/p$i.log" 2>&1 \
      || { echo "pass $i rc=$?" >> "$OUT/status.txt"; exit 20; }
done
echo done >> "$OUT/status.txt"
