#!/bin/bash
# Round profile set for the bench command (run on the GPU box):
#   1. bench.py itself (JSON line)                       -> $OUT/bench.json
#   2. rocprofv3 --kernel-trace --stats of the same run   -> $OUT/kt/
#   3. rocprofv3 --pmc WRITE_SIZE  (own pass)             -> $OUT/pmc_w/
#   4. rocprofv3 --pmc FETCH_SIZE  (own pass)             -> $OUT/pmc_f/
# Usage: tools/profile_round.sh <outdir> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1; shift
ARGS="$@"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 900 python3 "$R/bench.py" $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 11
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- \
    python3 "$R/bench.py" $ARGS --no-cpu-baseline > "$OUT/kt.log" 2>&1 || exit 12
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_w" -o pmc -- \
    python3 "$R/bench.py" $ARGS --no-cpu-baseline > "$OUT/pmc_w.log" 2>&1 || exit 13
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_f" -o pmc -- \
    python3 "$R/bench.py" $ARGS --no-cpu-baseline > "$OUT/pmc_f.log" 2>&1 || exit 14
echo ok > "$OUT/done"
