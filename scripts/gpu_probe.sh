#!/bin/bash
# One-call GPU probe: selected parity tests (PROBE_K, a pytest -k expression
# over the decode / list / fuzz / regex GPU tests), then A/B lines of
# scripts/ab_opts.py: each further argument is one "CONFIG ROWS VARIANT..."
# string.  Every GPU step has its own time limit; the first failure ends it.
set -o pipefail
TAG=${1:?tag}
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$PROBE_K" ]; then
    timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_lists.py tests/test_gpu_fuzz.py \
        tests/test_gpu_regex.py tests/test_gpu_cpp_api.py tests/test_gpu_c3_full.py -m gpu -k "$PROBE_K" -x -q --timeout 120 --timeout-method thread \
        > "$OUT/pytest_probe.log" 2>&1
    rc=$?; tail -5 "$OUT/pytest_probe.log"
    [ $rc -eq 0 ] || { echo "PYTEST rc=$rc"; exit $rc; }
fi
i=0
for ab in "$@"; do
    i=$((i + 1))
    timeout -k 10 300 python3 scripts/ab_opts.py $ab > "$OUT/ab_$i.txt" 2>&1
    rc=$?; echo "== $ab"; cat "$OUT/ab_$i.txt"; [ $rc -eq 0 ] || exit $rc
done
echo PROBE_OK
