#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-rxabl}; mkdir -p "$OUT"; export TMPDIR=/tmp
for d in 0 1 2 3; do
  PQ_OPTS=regex_debug=$d timeout -k 10 200 python scripts/regex_ab.py "special.*requests" "[0-9]" > "$OUT/d$d.json" 2>&1 || { cat "$OUT/d$d.json"; exit 1; }
  echo "debug=$d"; cat "$OUT/d$d.json"
done
