#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r6f}; mkdir -p "$OUT"
timeout -k 10 400 python scripts/ab_opts.py C2 10000000 - write_ilv=1 write_ilv=1,write_waves=8 write_ilv=1,write_waves=16 > "$OUT/ab.txt" 2>&1
rc=$?; cat "$OUT/ab.txt"; exit $rc
