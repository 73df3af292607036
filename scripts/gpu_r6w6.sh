#!/bin/bash
# round 6: C2 end to end, host walk vs device walk (bench e2e leg), C3 regex end to end
set -o pipefail
OUT=gpurun_out/${1:-r6w6}; mkdir -p "$OUT"
timeout -k 10 600 python bench.py --no-cpu --no-c4 --no-c5 --no-ext --no-wide --steps 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit $rc; }
cp gpurun_out/bench_full.json "$OUT/bench_full.json"
python3 - <<'PY'
import json
d = json.load(open('gpurun_out/bench_full.json'))
e = d['end_to_end']['c2']
dw = e.get('device_walk', {})
print('c2 host-walked total', round(e['total_ms'], 3), 'upload', round(e['upload_ms'], 3), 'walk', e['upload_phases']['up_walk'])
print('c2 device-walked total', round(dw.get('total_ms', 0), 3), 'upload', round(dw.get('upload_ms', 0), 3), 'walk', dw.get('upload_phases', {}).get('up_walk'))
c3 = d['end_to_end'].get('c3_regex') or d['end_to_end'].get('c3')
print('c3', json.dumps(c3)[:300] if c3 else None)
PY
