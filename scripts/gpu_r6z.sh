#!/bin/bash
# round 6: the codec parsers moved to lz.hpp / deflate.hpp: codec GPU tests and the bench's codec legs
set -o pipefail
OUT=gpurun_out/${1:-r6z}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ext.py tests/test_gpu_fuzz.py -m gpu -q --timeout=300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu --no-c4 --no-c5 --no-wide --no-e2e --no-regex --steps 10 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit $rc; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_full.json')); e=d.get('ext') or {}
print(json.dumps({k: (v.get('codec_GBs_out') if isinstance(v, dict) else v) for k, v in e.items()})[:800])"
