#!/usr/bin/env python3
"""k_wide_rows phase clocks on bench.py's wide-dictionary column (option
"fused_prof"): thread 0's shader-clock time per phase, per page, averaged
over the decodes.  usage: wide_prof.py [rows]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
from pqgpu import capi, gen  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
col = gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=0.05, dict_size=100_000,
              len_min=4, len_max=9, max_run=16)
f = gen.build([col], rows, 1, seed=gen.CONFIG_SEEDS["C2"], layout=gen.ARROW_LAYOUT)
ctx = capi.Context(0)
dc = ctx.upload(f, [capi.File(f).chunk(0, 0)])
dc.decode()
ctx.set_option("fused_prof", 1)
ctx.fused_prof_read(raw=True)
for _ in range(5):
    dc.decode()
v = ctx.fused_prof_read(raw=True)
names = ["stage+prologue", "def spec", "def expand", "ranks", "index spec", "rows", "fallback pages", "pages"]
pages = max(v[7], 1)
print(json.dumps({"pages": v[7], "fallback_pages": v[6],
                  "clocks_per_page": {names[i]: round(v[i] / pages) for i in range(6)}}))
