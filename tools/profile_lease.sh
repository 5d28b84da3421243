#!/bin/bash
# Round-4 profile set (run on the GPU box from the repo root):
#   bench.json            the N = 1 bench line (config 3 + its config5 object + cpu_baseline)
#   bench_{kt,w,f}/       rocprofv3 --kernel-trace --stats / --pmc WRITE_SIZE / --pmc FETCH_SIZE
#                         of the same bench command (separate passes, MI355X_MICROARCH.md)
#   band_{v,h}_{kt,w,f}/  the same three passes over one config-4 rank's band filled alone
#                         (tools/band_alone.py --rank 7, vertical / horizontal sweep)
# then: python tools/summarize_r04.py <outdir> <tag>
# Usage: bash tools/profile_lease.sh <outdir>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
B="python3 $R/bench.py --steps 10 --warmup 3"
timeout -k 10 400 $B > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 11
for pass in "kt:--kernel-trace --stats" "w:--pmc WRITE_SIZE" "f:--pmc FETCH_SIZE"; do
  n=${pass%%:*}; a=${pass#*:}
  timeout -k 10 400 rocprofv3 $a --output-format csv -d "$OUT/bench_$n" -o p -- $B --no-cpu-baseline \
      > "$OUT/bench_$n.log" 2>&1 || exit 12
done
for sw in v:vertical h:horizontal; do
  s=${sw%%:*}; name=${sw#*:}
  for pass in "kt:--kernel-trace --stats" "w:--pmc WRITE_SIZE" "f:--pmc FETCH_SIZE"; do
    n=${pass%%:*}; a=${pass#*:}
    timeout -k 10 200 rocprofv3 $a --output-format csv -d "$OUT/band_${s}_$n" -o p -- \
        python3 "$R/tools/band_alone.py" --rank 7 --sweep $name --reps 3 > "$OUT/band_${s}_$n.log" 2>&1 || exit 13
  done
done
echo ok > "$OUT/done"
