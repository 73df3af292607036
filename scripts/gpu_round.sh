#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace + HBM PMC
# passes.  Every GPU step has its own time limit; the chain stops at the first
# failure (no retries).  Outputs land in gpurun_out/ (merged back by gpurun).
#   usage: bash scripts/gpu_round.sh [tag] [bench args...]
# The headline profile passes (prof_kt, prof_fetch, prof_write) run the C2
# decode and the C3 regex/decode legs only (--no-c4 --no-c5), so per-launch
# kernel averages and HBM bytes belong to the bench line's dominant kernel;
# prof_all traces every leg.
set -o pipefail
TAG=${1:-r1}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2)" | tee "$OUT/host.txt"

timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout=300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || { echo "PYTEST rc=$rc"; exit $rc; }

timeout -k 10 600 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; cat "$OUT/bench.json"; [ $rc -eq 0 ] || { echo "BENCH rc=$rc"; tail -20 "$OUT/bench.err"; exit $rc; }

HEAD_ARGS="--no-cpu --no-c4 --no-c5 --no-ext"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_kt" -o kt --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 $HEAD_ARGS "$@" > "$OUT/prof_kt.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "KT rc=$rc"; tail -20 "$OUT/prof_kt.log"; exit $rc; }

timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_all" -o all --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu "$@" > "$OUT/prof_all.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "KT-ALL rc=$rc"; tail -20 "$OUT/prof_all.log"; exit $rc; }

timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/prof_fetch" -o fetch --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 $HEAD_ARGS "$@" > "$OUT/prof_fetch.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "FETCH rc=$rc"; tail -20 "$OUT/prof_fetch.log"; exit $rc; }

timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/prof_write" -o write --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 $HEAD_ARGS "$@" > "$OUT/prof_write.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "WRITE rc=$rc"; tail -20 "$OUT/prof_write.log"; exit $rc; }
python3 scripts/pmc_summary.py "$OUT" "$OUT/pmc_summary.json" > /dev/null
cp "$OUT"/prof_kt/*kernel_stats.csv "$OUT/kernel_stats.csv"
cp "$OUT"/prof_all/*kernel_stats.csv "$OUT/kernel_stats_all_legs.csv"
echo ROUND_OK
