#!/bin/bash
# C2 writer shape A/Bs and the SQ counters of k_pipe_fused.
set -o pipefail
TAG=${1:-r4wr}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/ab_opts.py C2 10000000 - write_waves=16 write_waves=12 write_waves=8 write_waves=6 \
    "write_waves=16,write_bpc=1" > "$OUT/ab_c2_writer.txt" 2>&1
rc=$?; cat "$OUT/ab_c2_writer.txt"; [ $rc -eq 0 ] || exit $rc
PQ_OPTS=pipe_fused=1 bash scripts/pmc_sq.sh $TAG/sq_fused decode 10000000 3 > "$OUT/sq_fused.txt" 2>&1
rc=$?; grep -E "^k_|SQ_" "$OUT/sq_fused.txt" | grep -A17 "^k_pipe_fused"; [ $rc -eq 0 ] || exit $rc
echo WR_OK
