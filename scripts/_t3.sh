#!/bin/bash
# A/B of the tree's build against ab_base on C4 OPTIONAL DOUBLE (c3) and INT64 (c0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-t3}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q -k "opt or OPT or c4 or C4 or double or int" \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for col in c3; do
timeout -k 10 300 python scripts/ab_opts.py C4:$col 10000000 - fixed_fused=0 > "$OUT/ab_$col.json" 2>&1 || { cat "$OUT/ab_$col.json"; exit 1; }
cat "$OUT/ab_$col.json"
AB_PKG=ab_base timeout -k 10 300 python scripts/ab_opts.py C4:$col 10000000 - fixed_fused=0 > "$OUT/ab_base_$col.json" 2>&1 || { cat "$OUT/ab_base_$col.json"; exit 1; }
cat "$OUT/ab_base_$col.json"
done
