#!/bin/bash
# round 6: codec parity + A/B of the tree, then the exec-skip probe (ab_EXEC)
set -o pipefail
OUT=gpurun_out/${1:-r6t}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ext.py tests/test_gpu_codec_edge.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/codec_ab.py 10000000 - > "$OUT/codec_ab.txt" 2>&1
rc=$?; head -3 "$OUT/codec_ab.txt"; [ $rc -eq 0 ] || exit $rc
AB_PKG=ab_EXEC timeout -k 10 300 python scripts/codec_ab.py 10000000 - > "$OUT/EXEC.txt" 2>&1
rc=$?; echo EXEC; head -3 "$OUT/EXEC.txt"; exit $rc
