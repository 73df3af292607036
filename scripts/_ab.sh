#!/bin/bash
# A/B of context options on one column: bash scripts/_ab.sh TAG CONFIG VARIANT...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ab}; CFG=${2:-C2}; shift 2; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python scripts/ab_opts.py $CFG 10000000 "$@" > "$OUT/ab.json" 2>&1; rc=$?
cat "$OUT/ab.json"; exit $rc
