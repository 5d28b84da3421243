#!/bin/bash
# A/B of builds of libnwhip on one box, alternating A B .. A B .. (run from the repo root):
#   SW 64k fill (config 5's fill), SW strip 0 alone, config-4 rank-7 band alone
#   (horizontal), two chained horizontal bands of 524288 x 32768 on one GPU.
# Usage: bash tools/ab_libs.sh <outfile> <libA> <libB> [<libC> ...]
set -o pipefail
OUT=$1
shift
LIBS="$*"
: > "$OUT"
run() {  # lib, label, command...
    local lib=$1 lab=$2
    shift 2
    echo "[$lab] $*" >> "$OUT"
    NWHIP_LIB=$lib timeout -k 10 180 "$@" >> "$OUT" 2>&1 || { echo "FAILED rc=$? ($lab $*)" >> "$OUT"; exit 1; }
}
for pass in 1 2; do
    for lib in $LIBS; do
        lab="pass$pass $(basename "$lib")"
        run "$lib" "$lab" python -u tools/sw_attr.py --n1 65536 --n2 65536 --reps 5
        run "$lib" "$lab" python -u tools/sw_attr.py --reps 5
        run "$lib" "$lab" python -u tools/band_alone.py --rank 7 --sweep horizontal --reps 3
        run "$lib" "$lab" python -u tools/local_bands_time.py --P 2 --only horizontal --reps 3
        # AB_TRACE=1: the band's strip timeline too (hop, mean lag; the TRACE build of the kernel)
        if [ "${AB_TRACE:-0}" = 1 ]; then run "$lib" "$lab" python -u tools/tband_trace.py --n2 65536 ${AB_TRACE_ARGS:-}; fi
    done
done
echo done >> "$OUT"
