"""Regex scan timing by string-index mode on the C3 column (10M rows):
regex_index 2 (every scan walks and files the index: the bench's cold
metric), 0 (every scan walks, nothing filed), 1 after a filing scan (warm).
Timing only; the page sets are compared with the first scan's."""
import sys
import time

import numpy as np

sys.path.insert(0, "duckdb-parquet-parser_amd")
from pqgpu import capi, gen  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
f = gen.build(gen.c3_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C3"])
ctx = capi.Context(0)
dc = ctx.upload(f, [capi.File(f).chunk(0, 0)])
ref = dc.regex_pages("special.*requests", False)
for mode in (2, 0, 1, 2, 0, 1):
    ctx.set_option("regex_index", mode)
    if mode == 1:
        dc.regex_pages("special.*requests", False)  # files the index
    ctx.sync()
    n = 20
    t = time.perf_counter()
    for _ in range(n):
        got = dc.regex_pages("special.*requests", False)
    ms = (time.perf_counter() - t) / n * 1e3
    print(f"regex_index={mode}: {ms:.4f} ms/scan (sync per scan), same pages: {bool(np.array_equal(got, ref))}", flush=True)
