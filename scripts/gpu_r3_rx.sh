#!/bin/bash
# Regex kernels: parity (every kernel x pattern x case), then the C3 scans of
# this build against AB builds, interleaved twice.
set -o pipefail
TAG=${1:-r3rx}
AB_DIRS=${2:-ab_r3b}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_regex.py tests/test_gpu_cpp_api.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
    timeout -k 10 200 python scripts/regex_ab.py > "$OUT/rx_tree_$i.json" 2>&1 || exit 1
    for d in $AB_DIRS; do
        AB_PKG=$d timeout -k 10 200 python scripts/regex_ab.py > "$OUT/rx_${d}_$i.json" 2>&1 || exit 1
    done
done
tail -n 4 "$OUT"/rx_*.json
echo R3RX_OK
