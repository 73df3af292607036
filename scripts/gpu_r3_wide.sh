#!/bin/bash
# Round-3 check of the generic-path rows/gather and the small-LDS levels form:
# decode parity (every path), then one-call A/Bs on the wide-dictionary leg's
# column, C4's DOUBLE OPTIONAL column and C3's OPTIONAL string shape.
set -o pipefail
TAG=${1:-r3w}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_dict_shapes.py tests/test_gpu_regex.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ab_opts.py W 10000000 - wide_rows=0 gather_rows=0 > "$OUT/ab_wide.json" 2> "$OUT/ab_wide.err" || { tail "$OUT/ab_wide.err"; exit 1; }
cat "$OUT/ab_wide.json"
timeout -k 10 300 python scripts/ab_opts.py C4:c3 12500000 - levels_small=0 > "$OUT/ab_c4.json" 2> "$OUT/ab_c4.err" || { tail "$OUT/ab_c4.err"; exit 1; }
cat "$OUT/ab_c4.json"
for i in 1 2; do
    timeout -k 10 200 python scripts/regex_ab.py > "$OUT/rx_tree_$i.json" 2>&1 || exit 1
    AB_PKG=ab_base timeout -k 10 200 python scripts/regex_ab.py > "$OUT/rx_base_$i.json" 2>&1 || exit 1
done
tail -n 4 "$OUT"/rx_*.json
echo R3W_OK
