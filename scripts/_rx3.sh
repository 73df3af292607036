#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-rx3}; mkdir -p "$OUT"; export TMPDIR=/tmp
for o in "" "regex_direct=1" "regex_win=16384" "regex_direct=1,regex_win=16384"; do
  PQ_OPTS=$o timeout -k 10 200 python scripts/regex_ab.py "special.*requests" "[0-9]" "e" >> "$OUT/ab.json" 2>&1 || { cat "$OUT/ab.json"; exit 1; }
  echo "--- $o" >> "$OUT/ab.json"
done
cat "$OUT/ab.json"
