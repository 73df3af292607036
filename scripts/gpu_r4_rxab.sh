#!/bin/bash
# C3 regex A/B of library builds (abvar/libpqgpu_*.so): the bench's regex
# legs with the tree's build, then with each variant copied over it.
set -o pipefail
TAG=${1:-r4rxab}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-cpu --no-c4 --no-c5 --no-ext --no-wide --no-e2e --steps 10"
timeout -k 10 300 python bench.py $ARGS > "$OUT/base.json" 2> "$OUT/base.err"
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/base.err"; exit $rc; }
cp duckdb-parquet-parser_amd/pqgpu/libpqgpu.so "$OUT/.keep.so"
for v in "$@"; do
  cp "abvar/libpqgpu_$v.so" duckdb-parquet-parser_amd/pqgpu/libpqgpu.so
  timeout -k 10 300 python bench.py $ARGS > "$OUT/$v.json" 2> "$OUT/$v.err"
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/$v.err"; exit $rc; }
done
cp "$OUT/.keep.so" duckdb-parquet-parser_amd/pqgpu/libpqgpu.so
python3 - "$OUT" base "$@" <<'PY'
import json, sys
out = sys.argv[1]
for v in sys.argv[2:]:
    d = json.loads(open(f"{out}/{v}.json").read().strip().splitlines()[-1])
    r = d["regex"]
    print(v, "cold", round(r["ms_per_scan"], 4), round(r["kernel_ms"], 4), "warm", round(r["warm"]["ms_per_scan"], 4),
          round(r["warm"]["kernel_ms"], 4), {k: (round(p["kernel_ms"], 4), round(p["warm"]["kernel_ms"], 4), p["validated"]) for k, p in r["patterns"].items()})
PY
echo RXAB_OK
