#!/usr/bin/env python3
"""k_regex_plain time per pattern on C3 (10M rows), with a digest of the page
flags so that builds can be compared (AB_PKG = a directory holding another
build's pqgpu package).  usage: regex_ab.py [pattern ...]"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.environ.get("AB_PKG") or os.path.join(ROOT, "duckdb-parquet-parser_amd")]
import numpy as np  # noqa: E402
from pqgpu import capi, gen  # noqa: E402

pats = sys.argv[1:] or ["special.*requests", "^(carefully|quickly) ", "[0-9]", "e"]
ctx = capi.Context(0)
for kv in filter(None, os.environ.get("PQ_OPTS", "").split(",")):  # e.g. PQ_OPTS=regex_debug=1
    k, v = kv.split("=")
    ctx.set_option(k, int(v))
f = gen.build(gen.c3_cols(), 10_000_000, 1, seed=gen.CONFIG_SEEDS["C3"])
F = capi.File(f)
dc = ctx.upload(f, [F.chunk(0, 0)])
for pat in pats:
    flags = np.asarray(dc.regex_pages(pat))
    for _ in range(3):
        dc.regex_pages_async(pat, False)
    ctx.sync()
    meds = []
    for _ in range(5):
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(10):
            dc.regex_pages_async(pat, False)
        ctx.sync()
        ms, n = ctx.timing_get("regex_plain")
        ctx.timing(False)
        meds.append(ms / max(n, 1))
    print(json.dumps({"pkg": os.environ.get("AB_PKG", "tree"), "pattern": pat, "ms": round(float(np.median(meds)), 4),
                      "reported": int(flags.sum()),
                      "sha": hashlib.sha256(flags.astype(np.uint8).tobytes()).hexdigest()[:12]}), flush=True)
