#!/bin/bash
# round 6: codec tests (small/full layouts), writer interleave A/B, codec throughput
set -o pipefail
OUT=gpurun_out/${1:-r6g}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ext.py tests/test_gpu_segments.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ab_opts.py C2 10000000 - write_ilv=1 write_ilv=1,write_waves=8 > "$OUT/ab.txt" 2>&1
rc=$?; cat "$OUT/ab.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 8 --warmup 2 --repeats 3 --no-cpu --no-c4 --no-c5 --no-wide --no-e2e --no-regex > "$OUT/bench_ext.json" 2> "$OUT/bench_ext.err"
rc=$?; python3 -c "import json;d=json.load(open('gpurun_out/bench_full.json'));print(json.dumps({k:(v.get('codec_GBs_out'),v.get('codec_kernel_ms')) for k,v in d['ext'].items()}))"; exit $rc
