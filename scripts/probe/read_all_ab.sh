set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5u
timeout -k 10 200 python3 -c "
import sys; sys.path[:0]=['.','duckdb-parquet-parser_amd']
from pqgpu import gen
f=gen.build(gen.c2_cols(),10_000_000,1,seed=gen.CONFIG_SEEDS['C2'])
open('/tmp/c2.parquet','wb').write(f)
" || exit 1
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export PQGPU_AB_NOPREFAULT=1; else unset PQGPU_AB_NOPREFAULT; fi
  echo "noprefault=$v"; timeout -k 10 200 ./duckdb-parquet-parser_amd/pqgpu/api_check /tmp/c2.parquet time_read_all 0 0 5 /tmp/c2.dump || exit 1
done
