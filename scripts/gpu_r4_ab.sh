#!/bin/bash
# Round-4 A/Bs of context options on the C2 step (scripts/ab_opts.py: per-kernel
# HIP-event times, wall time, outputs checked equal to the first variant's).
set -o pipefail
TAG=${1:-r4ab}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 scripts/ab_opts.py C2 10000000 - pipe_run_pages=0 pipe_run_dict=0 pipe_run_pages=16 pipe_run_pages=8 \
    "pipe_run_pages=16,pipe_run_dict=0" fused_debug=67108864 > "$OUT/ab_c2_runs.txt" 2>&1
rc=$?; cat "$OUT/ab_c2_runs.txt"; [ $rc -eq 0 ] || exit $rc
echo AB_OK
