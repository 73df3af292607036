#!/usr/bin/env python3
"""Upload phases (host walk, plan sub-phases, allocation, H2D) of C2 and C3
from host file bytes, mean of 3 uploads each (timing table of pq_ctx)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.environ.get("AB_PKG") or os.path.join(ROOT, "duckdb-parquet-parser_amd")]
from pqgpu import capi, gen  # noqa: E402

PH = ("up_walk", "up_plan", "up_plan_pages", "up_plan_fused", "up_plan_pipe", "up_plan_plain", "up_plan_rest",
      "up_alloc", "up_h2d")
ctx = capi.Context(0)
REPS = int(os.environ.get("REPS", "3"))
CFGS = os.environ.get("CFGS", "C2,C3,C2a").split(",")
for name, cols, seed, layout in (("C2", gen.c2_cols(), 2, gen.REF_LAYOUT), ("C3", gen.c3_cols(), 3, gen.REF_LAYOUT),
                                 ("C2a", gen.c2_cols(), 2, gen.ARROW_LAYOUT)):
    if name not in CFGS:
        continue
    f = gen.build(cols, 10_000_000, 1, seed=seed, layout=layout)
    ch = capi.File(f).chunk(0, 0)
    x = ctx.upload(f, [ch])
    x.free()
    ctx.timing(True)
    ctx.timing_reset()
    walls = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        x = ctx.upload(f, [ch])
        ctx.sync()
        walls.append((time.perf_counter() - t0) * 1e3)
        x.free()
    ctx.timing(False)
    out = {k: round(ctx.timing_get(k)[0] / REPS, 3) for k in PH}
    print(json.dumps({"pkg": os.environ.get("AB_PKG", "tree"), "config": name,
                      "upload_ms": round(sorted(walls)[len(walls) // 2], 3), **out}), flush=True)
