#!/bin/bash
# One GPU call: decode parity tests, then A/B timings of the tree's build
# against the packages named in AB_DIRS (directories holding a pqgpu build),
# then one SQ-counter pass over the C2 decode and the C3 regex scan.
#   usage: bash scripts/gpu_ab.sh TAG "ab_base ab_b ..."
set -o pipefail
TAG=${1:-ab}
AB_DIRS=${2:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_regex.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for cfg in C2 C2a; do
    timeout -k 10 200 python scripts/ab_opts.py $cfg 10000000 - > "$OUT/dec_${cfg}_tree.json" 2>&1 || exit 1
    for d in $AB_DIRS; do
        AB_PKG=$d timeout -k 10 200 python scripts/ab_opts.py $cfg 10000000 - > "$OUT/dec_${cfg}_$d.json" 2>&1 || exit 1
    done
done
timeout -k 10 200 python scripts/regex_ab.py > "$OUT/rx_tree.json" 2>&1 || exit 1
for d in $AB_DIRS; do
    AB_PKG=$d timeout -k 10 200 python scripts/regex_ab.py > "$OUT/rx_$d.json" 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES \
    SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES -T -d "$OUT/sq" -o sq --output-format csv -- \
    python3 scripts/kernel_driver.py decode 10000000 3 > "$OUT/sq_dec.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES \
    SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES -T -d "$OUT/sqr" -o sqr --output-format csv -- \
    python3 scripts/kernel_driver.py regex 10000000 3 > "$OUT/sq_rx.log" 2>&1 || exit 1
echo done
