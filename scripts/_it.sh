#!/bin/bash
# iteration script: [decode/regex parity], then A/B timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-it}
TESTS=${2:-1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$TESTS" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_regex.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python scripts/ab_opts.py C2 10000000 - pipe_front=0 $AB_EXTRA > "$OUT/c2.json" 2>&1 || { cat "$OUT/c2.json"; exit 1; }
cat "$OUT/c2.json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 scripts/kernel_driver.py decode 10000000 5 > "$OUT/kt.log" 2>&1 || exit 1
grep -E "k_pipe|k_dict" "$OUT"/kt/*kernel_stats.csv | cut -d, -f1-4
echo IT_OK
