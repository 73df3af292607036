#!/bin/bash
# PMC passes over the C2 and C3-regex legs (no C4, C5, e2e or other legs, so
# k_regex_plain's per-launch bytes come from the C3 scans only): a kernel
# trace, then separate FETCH_SIZE and WRITE_SIZE passes, summarised by
# pmc_summary.py (corrections per MI355X_MICROARCH.md).
set -o pipefail
TAG=${1:-r4}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
C2_ARGS="--no-cpu --no-c4 --no-c5 --no-ext --no-wide --no-e2e --steps 10 --warmup 2 --repeats 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_kt" -o kt --output-format csv -- \
    python3 bench.py $C2_ARGS "$@" > "$OUT/prof_kt.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "KT rc=$rc"; tail -20 "$OUT/prof_kt.log"; exit $rc; }
cp "$OUT"/prof_kt/*kernel_stats.csv "$OUT/kernel_stats_rx.csv"
timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/prof_fetch" -o fetch --output-format csv -- \
    python3 bench.py $C2_ARGS "$@" > "$OUT/prof_fetch.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "FETCH rc=$rc"; tail -20 "$OUT/prof_fetch.log"; exit $rc; }
timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/prof_write" -o write --output-format csv -- \
    python3 bench.py $C2_ARGS "$@" > "$OUT/prof_write.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "WRITE rc=$rc"; tail -20 "$OUT/prof_write.log"; exit $rc; }
python3 scripts/pmc_summary.py "$OUT" "$OUT/pmc_rx.json" > /dev/null
echo PMC_RX_OK
