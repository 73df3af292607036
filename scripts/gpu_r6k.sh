#!/bin/bash
# round 6: regex prefilter parity + C3 scan timing
set -o pipefail
OUT=gpurun_out/${1:-r6k}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_regex.py tests/test_gpu_c3_full.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu --no-c4 --no-c5 --no-ext --no-wide --no-e2e --steps 10 > "$OUT/rx.json" 2> "$OUT/rx.err"
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/rx.err"; exit $rc; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench_full.json'));r=d['regex']
print('cold', r['ms_per_scan'], r['roofline_frac'], 'warm', r['warm']['ms_per_scan'], r['warm']['roofline_frac'], r['all_validated'])
print({k:(v.get('ms_per_scan'), v.get('warm',{}).get('ms_per_scan'), v.get('validated')) for k,v in r['patterns'].items()})"
