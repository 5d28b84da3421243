#!/bin/bash
# Leader-throttle sweep for a horizontal-strip band (run from the repo root): tband_trace on
# 524288 x 65536 with NW_LEAD_SLEEP = each value, two passes, for the given shape/poll args.
# Usage: bash tools/lead_sweep.sh <outfile> "<tband_trace args>" <sleep> [<sleep> ...]
set -o pipefail
OUT=$1
ARGS=$2
shift 2
: > "$OUT"
for pass in 1 2; do
    for ls in "$@"; do
        echo "[pass$pass NW_LEAD_SLEEP=$ls] tband_trace $ARGS" >> "$OUT"
        NW_LEAD_SLEEP=$ls timeout -k 10 150 python -u tools/tband_trace.py --n2 65536 $ARGS >> "$OUT" 2>&1 ||
            { echo "FAILED rc=$?" >> "$OUT"; exit 1; }
    done
done
echo done >> "$OUT"
