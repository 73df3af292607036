#!/bin/bash
# Regex round: the regex GPU tests (every kernel, full-size C3 page sets), the
# windowed kernel's phase ablation, then the bench's regex legs.
set -o pipefail
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_regex.py tests/test_gpu_c3_full.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert" "$OUT/pytest.log" | head -20; exit $rc; }
timeout -k 10 240 python3 scripts/regex_ablate.py > "$OUT/regex_ablate.txt" 2>&1
rc=$?; cat "$OUT/regex_ablate.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --no-c4 --no-c5 --no-ext --no-wide --no-e2e --steps 10 > "$OUT/rx.json" 2> "$OUT/rx.err"
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/rx.err"; exit $rc; }
python3 - "$OUT/rx.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["regex"]
print("c2", round(d["ms_per_step"], 4), "regex cold", round(r["ms_per_scan"], 4), round(r["kernel_ms"], 4), "warm",
      round(r["warm"]["ms_per_scan"], 4), round(r["warm"]["kernel_ms"], 4), "all_validated", r.get("all_validated"))
for k, p in r["patterns"].items():
    print(" ", k, round(p["kernel_ms"], 4), round(p["warm"]["kernel_ms"], 4), p["validated"])
PY
echo RX_OK
