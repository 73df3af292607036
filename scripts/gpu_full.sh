#!/bin/bash
# One GPU call for a round's evidence: the whole parity suite (no -x: every
# failure listed), the default bench line, a kernel trace of the headline
# legs, then the C2-only PMC passes (gpu_pmc_c2.sh).  Plain test failures
# (pytest rc 1) still go on to the measurements; a crash, abort or time limit
# of any step ends the call.
set -o pipefail
TAG=${1:-r5}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2)" | tee "$OUT/host.txt"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout=300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -15 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "PYTEST rc=$rc"; exit $rc; }
timeout -k 10 600 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; tail -c 400 "$OUT/bench.json"; [ $rc -eq 0 ] || { echo "BENCH rc=$rc"; tail -20 "$OUT/bench.err"; exit $rc; }
cp gpurun_out/bench_full.json "$OUT/bench_full.json"  # (the profiled runs below overwrite it)
HEAD_ARGS="--no-cpu --no-c4 --no-c5 --no-ext --no-wide"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_kt" -o kt --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 $HEAD_ARGS "$@" > "$OUT/prof_kt.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "KT rc=$rc"; tail -20 "$OUT/prof_kt.log"; exit $rc; }
cp "$OUT"/prof_kt/*kernel_stats.csv "$OUT/kernel_stats.csv"
bash scripts/gpu_pmc_c2.sh "$TAG"
rc=$?; [ $rc -eq 0 ] || exit $rc
# the wide dictionary pipe's kernels (bench leg `wide_dict`): their own trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_wide" -o kw --output-format csv -- \
    python3 scripts/ab_opts.py W 10000000 - > "$OUT/prof_wide.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "WIDE KT rc=$rc"; tail -20 "$OUT/prof_wide.log"; exit $rc; }
cp "$OUT"/prof_wide/*kernel_stats.csv "$OUT/kernel_stats_wide.csv"
echo done
