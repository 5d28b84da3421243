# final validation (tools/r04/k.sh) then the horizontal non-temporal store A/B (tools/r04/j.sh)
set -o pipefail
bash tools/r04/k.sh || exit $?
bash tools/r04/j.sh || exit $?
