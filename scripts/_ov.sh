#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ov}; mkdir -p "$OUT"; export TMPDIR=/tmp
shift
timeout -k 10 400 python scripts/overlap_probe.py 10000000 "$@" > "$OUT/ov.json" 2>&1; rc=$?
cat "$OUT/ov.json"; exit $rc
