#!/bin/bash
# round 6: where the two-wave codec's parser spends its time (probe builds ab_EXEC, ab_PUSH, ab_CHECK)
set -o pipefail
OUT=gpurun_out/${1:-r6s}; mkdir -p "$OUT"
for P in EXEC PUSH CHECK; do
  AB_PKG=ab_$P timeout -k 10 300 python scripts/codec_ab.py 10000000 - > "$OUT/$P.txt" 2>&1
  rc=$?; echo $P; head -3 "$OUT/$P.txt"; [ $rc -eq 0 ] || exit $rc
done
