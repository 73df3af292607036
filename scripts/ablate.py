#!/usr/bin/env python3
"""Ablation timings of the fused BYTE_ARRAY kernel (C2 shape) on one GPU.

fused_debug bits (timing only; the output is not valid with bits set):
  1 = skip the decoupled look-back (fake page bases)
  2 = skip the character gather
  4 = skip the offsets stores
  8 = writer: skip assembling the character blocks (stores zeros)
 16 = writer: assemble the character blocks but do not store them
 32 = writer: skip the block -> row map (wrong rows, same work otherwise)
Prints one JSON line per variant with per-kernel average milliseconds.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
from pqgpu import capi, gen  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
layout = gen.ARROW_LAYOUT if "arrow" in sys.argv else gen.REF_LAYOUT
f = gen.build(gen.c2_cols(), rows, 1, seed=2, layout=layout)
F = capi.File(f)
chunks = [F.chunk(0, 0)]
ctx = capi.Context(0)
variants = [(0, 0), (1, 0), (2, 0), (3, 0), (8, 0), (16, 0), (32, 0), (24, 0), (0, 8), (0, 4)]
for fused in (1, 0):
    for dbg, waves in (variants if fused else [(0, 0)]):
        ctx.set_option("fused_ba", fused)
        ctx.set_option("fused_debug", dbg)
        ctx.set_option("fused_waves", waves)
        dc = ctx.upload(f, chunks)
        dc.decode_async()
        ctx.sync()
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(10):
            dc.decode_async()
        ctx.sync()
        res = {}
        for k in ("dict_index", "dict_entries", "ba_fused", "ba_rows", "scan", "ba_gather"):
            ms, n = ctx.timing_get(k)
            if n:
                res[k] = round(ms / n, 4)
        ctx.timing(False)
        print(json.dumps({"fused": fused, "debug": dbg, "waves": waves, "ms": res}), flush=True)
        dc.free()
ctx.set_option("fused_debug", 0)
ctx.set_option("fused_waves", 0)
# per-phase shader clocks of the fused kernel (cycles per page, summed over waves)
ctx.set_option("fused_ba", 1)
ctx.set_option("fused_prof", 1)
for dbg in (0, 1, 16):
    ctx.set_option("fused_debug", dbg)
    dc = ctx.upload(f, chunks)
    dc.decode_async()
    ctx.sync()
    ctx.fused_prof_read()
    for _ in range(5):
        dc.decode_async()
    ctx.sync()
    pr = ctx.fused_prof_read()
    pages = max(pr.get("pages", 1), 1)
    print(json.dumps({"debug": dbg, "prof_cycles_per_page": {k: round(v / pages, 1) for k, v in pr.items()
                                                             if k not in ("pages", "w_pages")},
                      "pages": pages, "w_pages": pr.get("w_pages")}), flush=True)
    dc.free()
ctx.set_option("fused_debug", 0)
ctx.set_option("fused_prof", 0)
