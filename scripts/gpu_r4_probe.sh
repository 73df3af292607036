#!/bin/bash
# Round-4 probe: parity of the new paths (k_pipe_fused "pfused", repeated
# columns, mutants), then A/Bs of k_pipe_fused and of k_pipe_runs' shape.
set -o pipefail
TAG=${1:-r4p}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_lists.py tests/test_gpu_fuzz.py tests/test_gpu_regex.py \
    -m gpu -k "${PROBE_K:-pfused or rep_ or lists or mutants}" ${PROBE_X--x} -q --timeout 120 --timeout-method thread > "$OUT/pytest_probe.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_probe.log"
# plain test failures (rc 1) may go on to the timings with PROBE_CONT=1; a
# crash, abort or time limit never does
[ $rc -eq 0 ] || [ $rc -eq 1 -a -n "$PROBE_CONT" ] || { echo "PYTEST rc=$rc"; exit $rc; }
timeout -k 10 300 python3 scripts/ab_opts.py W 10000000 pipe_wide=0 - > "$OUT/ab_wide.txt" 2>&1
rc=$?; cat "$OUT/ab_wide.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ab_opts.py C2 10000000 - pipe_fused=1 "pipe_fused=1,pipe_fused_waves=16" \
    "pipe_fused=1,pipe_fused_waves=4" pipe_run_pages=0 "pipe_fused=1,pipe_run_pages=0" > "$OUT/ab_c2.txt" 2>&1
rc=$?; cat "$OUT/ab_c2.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ab_opts.py C2 10000000 - pipe_run_pages=16 pipe_run_pages=8 pipe_run_dict=0 \
    fused_debug=67108864 > "$OUT/ab_c2_runs.txt" 2>&1
rc=$?; cat "$OUT/ab_c2_runs.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ab_opts.py C2a 10000000 - fused_debug=65536 fused_debug=131072 fused_debug=4096 fused_debug=8192 fused_debug=16384 \
    fused_debug=32768 > "$OUT/ab_c2a_big_phases.txt" 2>&1
rc=$?; cat "$OUT/ab_c2a_big_phases.txt"; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_sq.sh $TAG/sq_decode decode 10000000 3 > "$OUT/sq_decode.txt" 2>&1
rc=$?; tail -60 "$OUT/sq_decode.txt" | grep -E "^k_|SQ_(WAVES|INSTS_VALU|INSTS_LDS|LDS_BANK|WAVE_CYCLES|WAIT_INST_ANY|ACTIVE_INST_ANY) "; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_sq.sh $TAG/sq_regex regex 10000000 3 > "$OUT/sq_regex.txt" 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
echo PROBE_OK
