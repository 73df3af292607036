#!/bin/bash
# Regex kernel check + timing (C3 legs of bench.py) and the k_pipe_big
# step-5 diagnostics of the wide-dictionary pages.
set -o pipefail
TAG=${1:-r4x}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/probe_big_diag.py 2000000 > "$OUT/big_diag.txt" 2>&1
rc=$?; cat "$OUT/big_diag.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_regex.py -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/pytest_regex.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_regex.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu --no-c4 --no-c5 --no-ext --no-wide --no-e2e > "$OUT/bench_rx.json" 2> "$OUT/bench_rx.err"
rc=$?; tail -c 300 "$OUT/bench_rx.json"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_rx.err"; exit $rc; }
echo RX_OK
