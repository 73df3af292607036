#!/bin/bash
# GPU parity suite, then the upload-phase A/B against ab_base
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-chk}; mkdir -p gpurun_out/$T; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout=300 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/_up.sh $T/up > /dev/null 2>&1 || { echo UP_FAIL; exit 1; }
echo CHK2_OK
