#!/bin/bash
# SQ instruction counters of the C2 front per ablation level
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-sqab}; mkdir -p "$OUT"; export TMPDIR=/tmp
shift
for dbg in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY -T -d "$OUT/d$dbg" -o p --output-format csv -- \
      python3 scripts/kernel_driver.py decode 10000000 3 $dbg > "$OUT/d$dbg.log" 2>&1 || { echo "rc fail $dbg"; tail -5 "$OUT/d$dbg.log"; exit 1; }
done
python3 - "$OUT" "$@" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for dbg in sys.argv[2:]:
    agg = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(f"{out}/d{dbg}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_pipe_front" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(dbg, {k: round(v / max(n[k], 1) / 1e6, 3) for k, v in sorted(agg.items())})
PY
