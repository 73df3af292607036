#!/bin/bash
# upload phase A/B: tree vs AB_DIR alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-up}; mkdir -p "$OUT"; export TMPDIR=/tmp
for i in 1 2 3; do
  REPS=9 CFGS=C2,C3 timeout -k 10 200 python scripts/upload_phases.py >> "$OUT/ab.json" 2>&1 || exit 1
  AB_PKG=${2:-ab_base} REPS=9 CFGS=C2,C3 timeout -k 10 200 python scripts/upload_phases.py >> "$OUT/ab.json" 2>&1 || exit 1
done
cat "$OUT/ab.json"
