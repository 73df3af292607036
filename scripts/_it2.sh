#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-it}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dict_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -15 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/overlap_probe.py 10000000 1:1 1:1:pipe_front=0 2:2:pipe_front=0 4:2:pipe_front=0 8:2:pipe_front=0 4:4:pipe_front=0 2:2 4:2 8:2 > "$OUT/ov.json" 2>&1; rc=$?
cat "$OUT/ov.json"; exit $rc
