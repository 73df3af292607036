#!/bin/bash
# C5 row groups over two contexts: does the front of one row group overlap the
# write pass of another when the writer leaves room on each CU (write_bpc)?
set -o pipefail
TAG=${1:-r5ov}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "" "--opt write_bpc=1" "--opt write_bpc=1 --opt write_waves=8" "--c5-streams 1"; do
    timeout -k 10 300 python3 -u bench.py --no-cpu --no-regex --no-c4 --no-wide --no-ext --no-e2e \
        --steps 5 --repeats 3 --c5-rgs 6 $v > "$OUT/c5.json" 2> "$OUT/c5.err"
    rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 "$OUT/c5.err"; exit $rc; }
    python3 - "$OUT/c5.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for key in ("c5", "c5_ref"):
    c = d.get(key, {})
    print(sys.argv[2] or "default", "c2", round(d["ms_per_step"], 4), key,
          {k: c.get(k) for k in ("decode_values_per_s", "decode_ms", "kernel_ms_per_step", "streams")})
PY
done
