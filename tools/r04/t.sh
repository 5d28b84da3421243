set -o pipefail
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 120 tools/ubench/page_spread > $O/page_spread.txt 2>&1 || exit 10
echo done > $O/done
