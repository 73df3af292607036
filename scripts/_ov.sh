#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ov}; mkdir -p "$OUT"; export TMPDIR=/tmp
shift
timeout -k 10 300 python scripts/overlap_probe.py 10000000 "$@" > "$OUT/ov.json" 2>&1; rc=$?
cat "$OUT/ov.json"; [ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python scripts/overlap_probe.py 10000000 "$@" > "$OUT/ov16.json" 2>&1; rc=$?
echo "--- GPU_MAX_HW_QUEUES=16"; cat "$OUT/ov16.json"; exit $rc
