#!/bin/bash
# fixed-width OPTIONAL fused levels: parity then A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-t2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_shard.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for col in c3 c0; do
timeout -k 10 300 python scripts/ab_opts.py C4:$col 10000000 - fixed_fused=0 > "$OUT/ab_$col.json" 2>&1 || { cat "$OUT/ab_$col.json"; exit 1; }
cat "$OUT/ab_$col.json"
done
