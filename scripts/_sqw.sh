#!/bin/bash
# writer SQ counters (C2 decode, debug 0 and 2) and the upload A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-sqw}
bash scripts/pmc_sq.sh $T/d0 decode 10000000 3 0 > gpurun_out/$T.d0.txt 2>&1 || exit 1
bash scripts/pmc_sq.sh $T/d2 decode 10000000 3 2 > gpurun_out/$T.d2.txt 2>&1 || exit 1
bash scripts/_up.sh $T/up > /dev/null 2>&1 || exit 1
echo SQW_OK
