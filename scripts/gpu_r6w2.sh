#!/bin/bash
# round 6: device walk with the segment staged in LDS: parity, then the C2 / C3 end-to-end legs
set -o pipefail
OUT=gpurun_out/${1:-r6w2}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/walk_probe.py > "$OUT/walk_probe.txt" 2>&1
rc=$?; tail -20 "$OUT/walk_probe.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu --no-c4 --no-c5 --no-ext --no-wide --steps 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit $rc; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_full.json')); e=d.get('e2e',{}); print('e2e_c2', e.get('total_ms'), 'device_walk', e.get('device_walk',{}).get('total_ms'), e.get('upload_phases'), e.get('device_walk',{}).get('upload_phases'))
r=d.get('regex',{}).get('end_to_end') or d.get('regex',{}).get('e2e'); print('c3', json.dumps(r)[:600])"
