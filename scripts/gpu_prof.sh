#!/bin/bash
# The profiling half of gpu_full.sh, for a tree whose parity suite and bench
# line were just taken by gpu_final.sh: a kernel trace of the headline legs,
# then the C2-only kernel trace and PMC passes (gpu_pmc_c2.sh).
set -o pipefail
TAG=${1:-prof}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
HEAD_ARGS="--no-cpu --no-c4 --no-c5 --no-ext --no-wide"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_kt" -o kt --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 $HEAD_ARGS "$@" > "$OUT/prof_kt.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "KT rc=$rc"; tail -20 "$OUT/prof_kt.log"; exit $rc; }
cp "$OUT"/prof_kt/*kernel_stats.csv "$OUT/kernel_stats.csv"
tail -c 300 "$OUT/prof_kt.log"
bash scripts/gpu_pmc_c2.sh "$TAG"
