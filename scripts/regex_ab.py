#!/usr/bin/env python3
"""C3 regex page filter: the streaming kernel against the windowed kernel,
same page flags required, kernel times (HIP events) for a few patterns.
usage: regex_ab.py [rows]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
import numpy as np  # noqa: E402
from pqgpu import capi, gen  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
ctx = capi.Context(0)
f = gen.build(gen.c3_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C3"])
F = capi.File(f)
dc = ctx.upload(f, [F.chunk(0, 0)])
for pat in ("special.*requests", "e", "[0-9]", "^(carefully|quickly) "):
    res = {}
    flags = {}
    for name, stream in (("window", 0), ("stream", 1), ("window", 0), ("stream", 1)):
        ctx.set_option("regex_stream", stream)
        flags[name] = dc.regex_pages(pat, False)
        for _ in range(3):
            dc.regex_pages_async(pat, False)
        ctx.sync()
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(10):
            dc.regex_pages_async(pat, False)
        ctx.sync()
        k = "regex_stream" if stream else "regex_plain"
        res[name] = round(ctx.timing_get(k)[0] / 10, 4)
        ctx.timing(False)
    same = bool(np.array_equal(flags["window"], flags["stream"]))
    print(json.dumps({"pattern": pat, "ms": res, "same": same, "reported": int(flags["stream"].sum()),
                      "pages": int(len(flags["stream"]))}), flush=True)
ctx.set_option("regex_stream", 1)
