#!/bin/bash
# First half of a round's GPU session: parity suite, default bench, kernel trace of the headline legs.
set -o pipefail
TAG=${1:-r3}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2)" | tee "$OUT/host.txt"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout=300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || { echo "PYTEST rc=$rc"; exit $rc; }
timeout -k 10 600 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; tail -c 400 "$OUT/bench.json"; [ $rc -eq 0 ] || { echo "BENCH rc=$rc"; tail -20 "$OUT/bench.err"; exit $rc; }
HEAD_ARGS="--no-cpu --no-c4 --no-c5 --no-ext --no-wide"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_kt" -o kt --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 $HEAD_ARGS "$@" > "$OUT/prof_kt.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "KT rc=$rc"; tail -20 "$OUT/prof_kt.log"; exit $rc; }
cp "$OUT"/prof_kt/*kernel_stats.csv "$OUT/kernel_stats.csv"
echo ROUND_A_OK
