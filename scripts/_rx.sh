#!/bin/bash
# regex parity, then per-pattern k_regex_plain A/B of the tree against ab_base
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-rx}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_regex.py tests/test_gpu_dict_shapes.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/regex_ab.py "special.*requests" "^(carefully|quickly) " "[0-9]" "e" > "$OUT/tree.json" 2>&1 || { cat "$OUT/tree.json"; exit 1; }
AB_PKG=ab_base timeout -k 10 200 python scripts/regex_ab.py "special.*requests" "^(carefully|quickly) " "[0-9]" "e" > "$OUT/base.json" 2>&1 || { cat "$OUT/base.json"; exit 1; }
cat "$OUT/tree.json" "$OUT/base.json"
