#!/bin/bash
# Wide-dictionary and k_pipe_big probe: the W column (100k-entry dictionary,
# 20,000-row pages of ~25 KiB: the two-segment jump table) with the wide pipe
# on / off and k_pipe_big's phase ablations; C2a (one segment) beside it.
set -o pipefail
TAG=${1:-r4w}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/ab_opts.py W 10000000 pipe_wide=0 - fused_debug=65536 fused_debug=4096 \
    fused_debug=8192 fused_debug=16384 fused_debug=32768 > "$OUT/ab_wide.txt" 2>&1
rc=$?; cat "$OUT/ab_wide.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ab_opts.py C2a 10000000 - fused_debug=65536 fused_debug=131072 fused_debug=4096 \
    fused_debug=8192 fused_debug=16384 fused_debug=32768 > "$OUT/ab_c2a.txt" 2>&1
rc=$?; cat "$OUT/ab_c2a.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ab_opts.py C2 10000000 - pipe_fused=1 "pipe_fused=1,pipe_fused_waves=4" > "$OUT/ab_c2.txt" 2>&1
rc=$?; cat "$OUT/ab_c2.txt"; [ $rc -eq 0 ] || exit $rc
echo WIDE_OK
