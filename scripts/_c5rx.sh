#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-c5rx}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_regex.py tests/test_gpu_dict_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu --no-regex --no-c4 --no-ext --no-wide --steps 8 > "$OUT/b.json" 2> "$OUT/b.err" || { tail "$OUT/b.err"; exit 1; }
python3 -c "
import json;d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1])
print('C2',d['value']/1e9,d['ms_per_step'])
for k in ('c5','c5_ref'):
  c=d[k];print(k,round(c['decode_ms'],4),round(c['regex_ms'],4),round(c['step_ms'],4),round(c['step_over_decode'],3),c['regex_validated'],{a:round(b,4) for a,b in c['kernel_ms_per_step'].items()})
"
