#!/usr/bin/env python3
"""C3 regex page filter: kernel time vs the windowed kernel's window bytes
(option regex_win) for a few patterns.  usage: regex_sweep.py [rows]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
from pqgpu import capi, gen  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
ctx = capi.Context(0)
f = gen.build(gen.c3_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C3"])
F = capi.File(f)
dc = ctx.upload(f, [F.chunk(0, 0)])
ref = {}
for win in [int(w) for w in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["8192", "4096", "2048", "16384"])]:
    ctx.set_option("regex_win", win)
    for pat in ("special.*requests", "e", "[0-9]"):
        flags = dc.regex_pages(pat)
        if pat in ref:
            assert (flags == ref[pat]).all(), (win, pat)
        ref[pat] = flags
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(5):
            dc.regex_pages_async(pat)
        ctx.sync()
        ms, n = ctx.timing_get("regex_plain")
        ctx.timing(False)
        dc.regex_pages_result()
        print(json.dumps({"win": win, "pattern": pat, "ms": round(ms / max(n, 1), 4), "reported": int(flags.sum())}),
              flush=True)
