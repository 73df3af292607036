#!/bin/bash
# Round-5 GPU call: the GPU suite, the regex ablation and bench legs, the
# C2 front A/B and the C5 stream-overlap probe.  Every GPU step has its own
# time limit and the first failure ends the call.
set -o pipefail
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$NO_SUITE" ]; then
    timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
    rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "PYTEST rc=$rc"; exit $rc; }
fi
timeout -k 10 120 python3 scripts/h2d_probe.py > "$OUT/h2d.json" 2>&1
rc=$?; cat "$OUT/h2d.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 scripts/regex_ablate.py > "$OUT/regex_ablate.txt" 2>&1
rc=$?; cat "$OUT/regex_ablate.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --no-c4 --no-c5 --no-ext --no-wide --no-e2e --steps 10 > "$OUT/rx.json" 2> "$OUT/rx.err"
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/rx.err"; exit $rc; }
python3 - "$OUT/rx.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["regex"]
print("c2", round(d["ms_per_step"], 4), "regex cold", round(r["ms_per_scan"], 4), round(r["kernel_ms"], 4), "warm",
      round(r["warm"]["ms_per_scan"], 4), round(r["warm"]["kernel_ms"], 4))
for k, p in r["patterns"].items():
    print(" ", k, round(p["kernel_ms"], 4), round(p["warm"]["kernel_ms"], 4), p["validated"])
PY
[ -n "$NO_AB" ] || bash scripts/gpu_probe.sh "$TAG" "C2 10000000 - pipe_front=1 pipe_front=1,win_pages=4,win_bytes=2048" || exit 1
[ -n "$NO_OV" ] || bash scripts/gpu_c5_overlap.sh "${TAG}ov" || exit 1
echo R5K_OK
