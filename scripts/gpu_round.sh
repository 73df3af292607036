#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace + HBM PMC
# passes.  Every GPU step has its own time limit; the chain stops at the first
# failure (no retries).  Outputs land in gpurun_out/ (merged back by gpurun).
#   usage: bash scripts/gpu_round.sh [tag] [bench args...]
set -o pipefail
TAG=${1:-r1}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2)" | tee "$OUT/host.txt"

timeout -k 10 900 python -m pytest tests -m gpu -q --timeout=300 > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || { echo "PYTEST rc=$rc"; exit $rc; }

timeout -k 10 600 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; cat "$OUT/bench.json"; [ $rc -eq 0 ] || { echo "BENCH rc=$rc"; tail -20 "$OUT/bench.err"; exit $rc; }

timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_kt" -o kt --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu "$@" > "$OUT/prof_kt.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "KT rc=$rc"; tail -20 "$OUT/prof_kt.log"; exit $rc; }

timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/prof_fetch" -o fetch --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu "$@" > "$OUT/prof_fetch.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "FETCH rc=$rc"; tail -20 "$OUT/prof_fetch.log"; exit $rc; }

timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/prof_write" -o write --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu "$@" > "$OUT/prof_write.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "WRITE rc=$rc"; tail -20 "$OUT/prof_write.log"; exit $rc; }
python3 scripts/pmc_summary.py "$OUT" "$OUT/pmc_summary.json" > /dev/null
cp "$OUT"/prof_kt/*kernel_stats.csv "$OUT/kernel_stats.csv"
echo ROUND_OK
