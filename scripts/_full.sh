#!/bin/bash
# full GPU suite then the default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-full}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout=300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; tail -c 300 "$OUT/bench.json"; [ $rc -eq 0 ] || { tail -20 "$OUT/bench.err"; exit $rc; }
