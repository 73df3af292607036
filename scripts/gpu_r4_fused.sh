#!/bin/bash
# k_pipe_fused bring-up: its parity tests (the "pfused" decode path), then
# A/Bs against the three-kernel pipe on C2 and C2a.
set -o pipefail
TAG=${1:-r4f}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_dict_shapes.py tests/test_gpu_lists.py \
    -m gpu -k "pfused" -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_pfused.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_pfused.log"; [ $rc -eq 0 ] || { echo "PYTEST rc=$rc"; exit $rc; }
timeout -k 10 300 python3 scripts/ab_opts.py C2 10000000 - pipe_fused=1 "pipe_fused=1,pipe_fused_waves=16" \
    "pipe_fused=1,pipe_fused_waves=4" > "$OUT/ab_c2_fused.txt" 2>&1
rc=$?; cat "$OUT/ab_c2_fused.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ab_opts.py C2a 10000000 - pipe_fused=1 > "$OUT/ab_c2a_fused.txt" 2>&1
rc=$?; cat "$OUT/ab_c2a_fused.txt"; [ $rc -eq 0 ] || exit $rc
echo FUSED_OK
