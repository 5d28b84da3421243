set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 60 tools/ubench/wave_simd > $O/wave_simd.txt 2>&1 || exit 10
echo done > $O/done
