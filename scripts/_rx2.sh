#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-rx2}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_regex.py tests/test_gpu_dict_shapes.py tests/test_gpu_shard.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
P='special.*requests ^(carefully|quickly)  [0-9] e'
timeout -k 10 200 python scripts/regex_ab.py "special.*requests" "^(carefully|quickly) " "[0-9]" "e" > "$OUT/tree.json" 2>&1 || { cat "$OUT/tree.json"; exit 1; }
PQ_OPTS=regex_index=0 timeout -k 10 200 python scripts/regex_ab.py "special.*requests" "e" > "$OUT/noidx.json" 2>&1 || { cat "$OUT/noidx.json"; exit 1; }
AB_PKG=ab_base timeout -k 10 200 python scripts/regex_ab.py "special.*requests" "^(carefully|quickly) " "[0-9]" "e" > "$OUT/base.json" 2>&1 || { cat "$OUT/base.json"; exit 1; }
cat "$OUT/tree.json" "$OUT/noidx.json" "$OUT/base.json"
