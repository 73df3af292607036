#!/bin/bash
# Wide rows: parity (decode, dictionary shapes), then the W column on this
# build against AB builds (AB_DIRS), interleaved twice.
set -o pipefail
TAG=${1:-r3w2}
AB_DIRS=${2:-ab_j16}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_dict_shapes.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
    timeout -k 10 300 python scripts/ab_opts.py W 10000000 - > "$OUT/w_tree_$i.json" 2>&1 || exit 1
    for d in $AB_DIRS; do
        AB_PKG=$d timeout -k 10 300 python scripts/ab_opts.py W 10000000 - > "$OUT/w_${d}_$i.json" 2>&1 || exit 1
    done
done
tail -n 2 "$OUT"/w_*.json
timeout -k 10 200 python scripts/wide_prof.py > "$OUT/wide_prof.json" 2>&1 || { tail "$OUT/wide_prof.json"; exit 1; }
cat "$OUT/wide_prof.json"
echo R3W2_OK
