#!/bin/bash
# round 6: k_pipe_page parity (decode paths default/runs, segments, regex over codes) and the C2 A/B
set -o pipefail
OUT=gpurun_out/${1:-r6c}; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_decode.py tests/test_gpu_regex.py -x -q \
    -k "not serial and not generic and not fused" --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -5 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ab_opts.py C2 10000000 - pipe_page=0 pipe_segs=2 pipe_segs=4 > "$OUT/ab.txt" 2>&1
rc=$?; cat "$OUT/ab.txt"; exit $rc
