#!/bin/bash
# SQ instruction/wait counters for the kernels of scripts/kernel_driver.py.
#   usage: bash scripts/pmc_sq.sh TAG [driver args...]
set -o pipefail
TAG=${1:-sq}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -T -d "$OUT/p$i" -o p$i --output-format csv -- \
      python3 scripts/kernel_driver.py "$@" > "$OUT/p$i.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "PMC pass $i rc=$rc"; tail -20 "$OUT/p$i.log"; exit $rc; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {v:16.0f}  (dispatches {cnt[(k, c)]})")
PY
