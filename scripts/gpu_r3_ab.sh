#!/bin/bash
# Full GPU parity suite, then one-call A/Bs of this build against AB_DIRS on
# the wide-dictionary column (W) and C4's DOUBLE OPTIONAL column, interleaved.
set -o pipefail
TAG=${1:-r3ab}
AB_DIRS=${2:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
    for cfg in W C4:c3; do
        n=10000000; [ $cfg = C4:c3 ] && n=12500000
        timeout -k 10 300 python scripts/ab_opts.py $cfg $n - > "$OUT/${cfg/:/_}_tree_$i.json" 2>&1 || exit 1
        for d in $AB_DIRS; do
            AB_PKG=$d timeout -k 10 300 python scripts/ab_opts.py $cfg $n - > "$OUT/${cfg/:/_}_${d}_$i.json" 2>&1 || exit 1
        done
    done
done
tail -n 1 "$OUT"/W_*.json "$OUT"/C4_c3_*.json
echo R3AB_OK
