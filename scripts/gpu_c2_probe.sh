#!/bin/bash
# C2 pipe anatomy in one GPU call: HBM write ceilings (torch fill / zero),
# then ab_opts variants of the three pipe kernels (ablation bits of
# fused_debug: 2 no characters, 4 no offsets/validity, 8 writer prologue only,
# 128 characters as aligned zero blocks, 1<<26 k_pipe_runs staging only), and
# the kernels' scaling with the row count.
set -o pipefail
TAG=${1:-c2p}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 120 python scripts/probe/write_bw.py > "$OUT/write_bw.txt" 2>&1 || exit $?
timeout -k 10 300 python scripts/ab_opts.py C2 10000000 - pipe_run_dict=0 fused_debug=67108864 fused_debug=128 \
    fused_debug=2 fused_debug=4 fused_debug=8 > "$OUT/ab_c2.txt" 2> "$OUT/ab_c2.err" || exit $?
timeout -k 10 200 python scripts/ab_opts.py C2 5000000 - > "$OUT/ab_c2_5m.txt" 2>&1 || exit $?
timeout -k 10 200 python scripts/ab_opts.py C2 2500000 - > "$OUT/ab_c2_2m5.txt" 2>&1 || exit $?
cat "$OUT"/write_bw.txt "$OUT"/ab_c2*.txt
