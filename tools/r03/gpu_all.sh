#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r03/dropin_time.sh && bash tools/r03/gputest.sh
