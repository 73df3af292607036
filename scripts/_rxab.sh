#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-rxab}; mkdir -p "$OUT"; export TMPDIR=/tmp
shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_regex.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/regex_ab.py "$@" > "$OUT/tree.json" 2>&1 || { cat "$OUT/tree.json"; exit 1; }
AB_PKG=ab_base timeout -k 10 200 python scripts/regex_ab.py "$@" > "$OUT/base.json" 2>&1 || { cat "$OUT/base.json"; exit 1; }
cat "$OUT/tree.json" "$OUT/base.json"
