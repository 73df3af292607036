#!/bin/bash
# PMC passes over the wide-dictionary decode (scripts/ab_opts.py W: the
# bench's wide_dict column, 10M rows, repeated decodes): a kernel trace, then
# separate FETCH_SIZE and WRITE_SIZE passes, summarised by pmc_summary.py.
set -o pipefail
TAG=${1:-r4}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
W_CMD="scripts/ab_opts.py W 10000000 -"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_kt" -o kt --output-format csv -- \
    python3 $W_CMD > "$OUT/prof_kt.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "KT rc=$rc"; tail -20 "$OUT/prof_kt.log"; exit $rc; }
cp "$OUT"/prof_kt/*kernel_stats.csv "$OUT/kernel_stats_w.csv"
timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/prof_fetch" -o fetch --output-format csv -- \
    python3 $W_CMD > "$OUT/prof_fetch.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "FETCH rc=$rc"; tail -20 "$OUT/prof_fetch.log"; exit $rc; }
timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/prof_write" -o write --output-format csv -- \
    python3 $W_CMD > "$OUT/prof_write.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "WRITE rc=$rc"; tail -20 "$OUT/prof_write.log"; exit $rc; }
python3 scripts/pmc_summary.py "$OUT" "$OUT/pmc_w.json" > /dev/null
echo PMC_W_OK
