#!/bin/bash
# round 6: C2 pipe A/B of launch shapes
set -o pipefail
OUT=gpurun_out/${1:-r6e}; mkdir -p "$OUT"
timeout -k 10 400 python scripts/ab_opts.py C2 10000000 - pipe_run_dict=0 pipe_run_pages=16 pipe_run_pages=0 write_waves=8 write_waves=16 write_waves=8,write_bpc=2 pipe_run_dict=0,write_waves=8 > "$OUT/ab.txt" 2>&1
rc=$?; cat "$OUT/ab.txt"; exit $rc
