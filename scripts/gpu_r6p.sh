#!/bin/bash
# round 6: SNAPPY parse-only probe (ab_probe built with PQ_CODEC_PARSE_ONLY=1) vs the full decode
set -o pipefail
OUT=gpurun_out/${1:-r6p}; mkdir -p "$OUT"
true

AB_PKG=ab_probe timeout -k 10 600 python scripts/codec_ab.py 10000000 - > "$OUT/parse_only.txt" 2>&1
rc=$?; cat "$OUT/parse_only.txt"; exit $rc
