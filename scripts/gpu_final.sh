#!/bin/bash
# The round's closing check: the whole parity suite, smoke(), the default bench line.
set -o pipefail
OUT=gpurun_out/${1:-final}; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout=300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -4 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; tail -c 600 "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/bench_full.json "$OUT/bench_full.json"
