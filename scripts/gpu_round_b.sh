#!/bin/bash
# Second half: kernel trace of every leg, then separate FETCH_SIZE / WRITE_SIZE
# PMC passes over the headline legs (no trace domains beside --pmc).
set -o pipefail
TAG=${1:-r3}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
HEAD_ARGS="--no-cpu --no-c4 --no-c5 --no-ext --no-wide"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_all" -o all --output-format csv -- \
    python3 bench.py --steps 6 --warmup 2 --repeats 3 --no-cpu "$@" > "$OUT/prof_all.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "KT-ALL rc=$rc"; tail -20 "$OUT/prof_all.log"; exit $rc; }
cp "$OUT"/prof_all/*kernel_stats.csv "$OUT/kernel_stats_all_legs.csv"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/prof_fetch" -o fetch --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --repeats 2 $HEAD_ARGS "$@" > "$OUT/prof_fetch.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "FETCH rc=$rc"; tail -20 "$OUT/prof_fetch.log"; exit $rc; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/prof_write" -o write --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --repeats 2 $HEAD_ARGS "$@" > "$OUT/prof_write.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "WRITE rc=$rc"; tail -20 "$OUT/prof_write.log"; exit $rc; }
python3 scripts/pmc_summary.py "$OUT" "$OUT/pmc_summary.json" > /dev/null
echo ROUND_B_OK
