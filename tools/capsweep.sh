set -o pipefail
for v in "" cap8 cap16 cap24 cap32; do
  if [ -n "$v" ]; then export NWHIP_LIB=$PWD/fast-needleman-wunsch_amd/build/libnwhip_$v.so; else unset NWHIP_LIB; fi
  echo "== variant ${v:-base}"
  timeout -k 10 200 python tools/quick_time.py --sizes 131072,262144 --waves 0 --sub 1,2 --reps 2 || exit 1
done
unset NWHIP_LIB
echo "== trace base"; timeout -k 10 200 python tools/trace_strips.py --n 262144 --waves 0 --sub 1 || exit 1
export NWHIP_LIB=$PWD/fast-needleman-wunsch_amd/build/libnwhip_cap16.so
echo "== trace cap16"; timeout -k 10 200 python tools/trace_strips.py --n 262144 --waves 0 --sub 1 || exit 1
