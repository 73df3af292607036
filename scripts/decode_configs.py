#!/usr/bin/env python3
"""Per-kernel decode timings for the SURVEY §8d configs C3 (PLAIN BYTE_ARRAY)
and C4 (mixed INT64/DOUBLE/dict/plain, one 10M-row row group per column) on
one GPU.  usage: decode_configs.py [rows] [config[:column],...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
from pqgpu import capi, gen  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
only = sys.argv[2].split(",") if len(sys.argv) > 2 else None  # e.g. "C4:c7,C3"
ctx = capi.Context(0)
KERNELS = ("dict_index", "dict_entries", "pipe_runs", "pipe_big", "plain_spec", "pipe_count", "pipe_codes", "pipe_write", "ba_fused", "ba_rows", "scan", "ba_gather", "fixed", "fixed_plain", "plain_ba")
for name, cols, layout, seed in [("C2", gen.c2_cols(), gen.REF_LAYOUT, 2),
                                 ("C2a", gen.c2_cols(), gen.ARROW_LAYOUT, 2),
                                 ("C3", gen.c3_cols(), gen.REF_LAYOUT, 3),
                                 ("C4", gen.c4_cols(), gen.ARROW_LAYOUT, 4)]:
    f = gen.build(cols, rows, 1, seed=seed, layout=layout)
    F = capi.File(f)
    for ci, c in enumerate(cols):
        if only and name not in only and f"{name}:{c.name}" not in only:
            continue
        dc = ctx.upload(f, [F.chunk(0, ci)])
        dc.decode()
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(5):
            dc.decode_async()
        ctx.sync()
        res = {k: round(ctx.timing_get(k)[0] / 5, 4) for k in KERNELS if ctx.timing_get(k)[1]}
        ctx.timing(False)
        tot = sum(res.values())
        print(json.dumps({"config": name, "col": c.name, "type": c.type, "pages": dc.num_pages,
                          "payload_MB": round(dc.payload_bytes / 1e6, 1), "ms": res,
                          "Gvalues_s": round(rows / (tot * 1e-3) / 1e9, 2) if tot else None}), flush=True)
        dc.free()
