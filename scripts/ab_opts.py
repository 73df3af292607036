#!/usr/bin/env python3
"""A/B of context options on one column: per-kernel times (HIP events), the
step's wall time without timers, and a byte-for-byte check of every variant's
output against the first variant's.
usage: ab_opts.py CONFIG[:col] [rows] VARIANT...
  VARIANT = "-" (defaults) or "key=value,key=value" (options set before upload)
  e.g. ab_opts.py C2 10000000 - big_all=1"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
import numpy as np  # noqa: E402
from pqgpu import capi, gen  # noqa: E402

CONFIGS = {"C2": (gen.c2_cols, gen.REF_LAYOUT, 2), "C2a": (gen.c2_cols, gen.ARROW_LAYOUT, 2),
           "C3": (gen.c3_cols, gen.REF_LAYOUT, 3), "C4": (gen.c4_cols, gen.ARROW_LAYOUT, 4)}
KERNELS = ("dict_index", "dict_entries", "pipe_runs", "pipe_big", "pipe_page", "plain_spec", "pipe_count", "pipe_codes",
           "pipe_write", "ba_batch", "ba_fused", "ba_rows", "scan", "ba_gather", "fixed", "fixed_plain", "plain_ba")

cfg, _, colname = sys.argv[1].partition(":")
rows = int(sys.argv[2])
variants = sys.argv[3:] or ["-"]
mk, layout, seed = CONFIGS[cfg]
cols = mk()
ci = next((i for i, c in enumerate(cols) if c.name == colname), 0) if colname else 0
f = gen.build(cols, rows, 1, seed=seed, layout=layout)
F = capi.File(f)
base = None
runs = []
for v in variants:
    ctx = capi.Context(0)
    opts = {} if v == "-" else {k: int(x) for k, x in (kv.split("=") for kv in v.split(","))}
    for k, x in opts.items():
        ctx.set_option(k, x)
    dc = ctx.upload(f, [F.chunk(0, ci)])
    dc.decode()
    h = dc.to_host()
    same = None
    if base is None:
        base = h
    else:
        same = bool(np.array_equal(h.validity, base.validity) and np.array_equal(h.data, base.data) and
                    (h.offsets is None or np.array_equal(h.offsets, base.offsets)))
    runs.append((v, ctx, dc, same))
# warm the clocks, then three alternating rounds (the median is reported)
for _ in range(100):
    runs[0][2].decode_async()
runs[0][1].sync()
res = {v: {"wall": [], "ms": []} for v, *_ in runs}
for rnd in range(3):
    for v, ctx, dc, same in runs:
        for _ in range(5):
            dc.decode_async()
        ctx.sync()
        steps = 50
        t0 = time.perf_counter()
        for _ in range(steps):
            dc.decode_async()
        ctx.sync()
        res[v]["wall"].append((time.perf_counter() - t0) / steps * 1e3)
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(10):
            dc.decode_async()
        ctx.sync()
        res[v]["ms"].append({k: ctx.timing_get(k)[0] / 10 for k in KERNELS if ctx.timing_get(k)[1]})
        ctx.timing(False)
for v, ctx, dc, same in runs:
    walls = sorted(res[v]["wall"])
    wall = walls[len(walls) // 2]
    ks = res[v]["ms"][0].keys()
    ms = {k: round(sorted(r[k] for r in res[v]["ms"])[1], 4) for k in ks}
    print(json.dumps({"variant": v, "same_as_first": same, "wall_ms": round(wall, 4),
                      "Gvalues_s": round(rows / wall / 1e6, 2), "ms": ms}), flush=True)
