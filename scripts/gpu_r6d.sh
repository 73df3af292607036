#!/bin/bash
# round 6: k_pipe_page phase timings (probe build) and SQ counters
set -o pipefail
OUT=gpurun_out/${1:-r6d}; mkdir -p "$OUT"
AB_PKG=ab_probe timeout -k 10 300 python scripts/ab_opts.py C2 10000000 - fused_debug=524288 fused_debug=1048576 fused_debug=2097152 fused_debug=4194304 pipe_page=0 > "$OUT/ab.txt" 2>&1
rc=$?; cat "$OUT/ab.txt"; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_sq.sh ${1:-r6d}/sq decode 10000000 3 > "$OUT/sq.txt" 2>&1
rc=$?; grep -A17 "k_pipe_page\|k_pipe_write" "$OUT/sq.txt" | head -40; exit $rc
