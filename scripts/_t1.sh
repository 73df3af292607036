#!/bin/bash
# targeted GPU tests + short bench (iteration script)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-t1}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_dict_shapes.py tests/test_gpu_regex.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "huge or dict_shapes or reuse or every_path or every_kernel or errors or crafted or regex_pages" > "$OUT/pytest.log" 2>&1
rc=$?; tail -15 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --no-cpu --no-regex --no-c4 --no-ext > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "
import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(d['value'],d['ms_per_step'],d['validated'])
print('c5',{k:v for k,v in d['c5'].items()})
print('wide',d['wide_dict'])
"
