#!/usr/bin/env python3
"""Windowed regex kernel phase ablation (option regex_debug): full, no DFA pass,
no chain walk, staging only, exact (serial) walk for every page; per window size.  Output flags are not valid
under the ablation.  usage: regex_ablate.py [win_bytes ...]"""
import json
import sys
import os
# AB_PKG: a directory holding another build's pqgpu package
sys.path[:0] = ["/root/repo", os.environ.get("AB_PKG") or "/root/repo/duckdb-parquet-parser_amd"]
from pqgpu import capi, gen  # noqa: E402
ctx = capi.Context(0)
# RX_INDEX=2: cold scans (every scan walks the length chains and files the index)
ctx.set_option("regex_index", int(os.environ.get("RX_INDEX", "1")))
f = gen.build(gen.c3_cols(), 10_000_000, 1, seed=gen.CONFIG_SEEDS["C3"])
F = capi.File(f)
for win in [int(a) for a in sys.argv[1:]] or [8192]:
    ctx.set_option("regex_win", win)
    dc = ctx.upload(f, [F.chunk(0, 0)])
    for dbg in [int(x) for x in os.environ.get("RX_DBG", "0,1,2,3,4").split(",")]:
        ctx.set_option("regex_debug", dbg)
        for _ in range(3):
            dc.regex_pages_async("special.*requests", False)
        ctx.sync()
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(10):
            dc.regex_pages_async("special.*requests", False)
        ctx.sync()
        ms, n = ctx.timing_get("regex_plain")
        ctx.timing(False)
        print(json.dumps({"win": win, "dbg": dbg, "index": int(os.environ.get("RX_INDEX", "1")), "ms": round(ms / n, 4),
                          "payload_frac_of_8TBs": round(dc.payload_bytes / (ms / n * 1e-3) / 8e12, 4)}), flush=True)
    ctx.set_option("regex_debug", 0)
    dc.free()
