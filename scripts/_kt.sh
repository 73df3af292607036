#!/bin/bash
# kernel traces of kernel_driver.py modes: bash scripts/_kt.sh tag "mode rows reps" ["mode rows reps" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for m in "$@"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt$i" -o kt --output-format csv -- python3 scripts/kernel_driver.py $m > "$OUT/kt$i.log" 2>&1 || { tail -5 "$OUT/kt$i.log"; exit 1; }
  echo "== $m"
  python3 - "$OUT/kt$i" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"  {r['Name'][:60]:60s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.2f}")
PY
done
echo KT_OK
