#!/bin/bash
# C3 regex A/B over options (bench.py's regex legs, each page set validated
# inside the bench): the default, then each "--opt k=v ..." group given.
set -o pipefail
TAG=${1:-r4rxopt}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-cpu --no-c4 --no-c5 --no-ext --no-wide --no-e2e --steps 10"
i=0
for v in "" "$@"; do
  opts=""
  for kv in $v; do opts="$opts --opt $kv"; done
  timeout -k 10 300 python bench.py $ARGS $opts > "$OUT/v$i.json" 2> "$OUT/v$i.err"
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/v$i.err"; exit $rc; }
  python3 - "$OUT/v$i.json" "${v:-default}" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["regex"]
print(sys.argv[2], "| cold", round(r["ms_per_scan"], 4), round(r["kernel_ms"], 4), "| warm", round(r["warm"]["ms_per_scan"], 4),
      round(r["warm"]["kernel_ms"], 4), "| all validated:", all(p["validated"] for p in r["patterns"].values()), "| C2", round(d["ms_per_step"], 4))
PY
  i=$((i+1))
done
echo RXOPT_OK
