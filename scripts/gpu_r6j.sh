#!/bin/bash
# round 6: C5 decode with the writer at 8 waves (co-residence with k_pipe_big on the other stream)
set -o pipefail
OUT=gpurun_out/${1:-r6j}; mkdir -p "$OUT"
for W in 10 8; do
  timeout -k 10 400 python bench.py --steps 4 --warmup 1 --repeats 3 --no-cpu --no-regex --no-c4 --no-wide --no-ext --no-e2e --no-c5-ref --opt write_waves=$W > "$OUT/c5_w$W.json" 2> "$OUT/c5_w$W.err"
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/c5_w$W.err"; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_full.json'));c=d['c5'];print($W, round(d['value']/1e9,2), round(c['decode_values_per_s']/1e9,2), c['kernel_ms_per_step'])"
done
