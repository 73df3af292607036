#!/bin/bash
# One GPU call for a round's evidence: the parity suite, the default bench
# line, a kernel trace of the headline legs (gpu_round_a.sh), then the C2-only
# PMC passes (gpu_pmc_c2.sh).  Stops at the first failing step.
set -o pipefail
TAG=${1:-r4}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_round_a.sh "$TAG" && bash scripts/gpu_pmc_c2.sh "$TAG"
