#!/usr/bin/env python3
"""Ablation timings of the fused BYTE_ARRAY kernel (C2 shape) on one GPU.

fused_debug bits (timing only; the output is not valid with bits set):
  1 = skip the decoupled look-back (fake page bases)
  2 = skip the character gather
  4 = skip the offsets stores
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
variants = [(0, 0), (1, 0), (2, 0), (3, 0), (7, 0), (0, 8), (0, 4), (0, 2), (3, 4)]
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
        for k in ("dict_index", "ba_fused", "ba_rows", "scan", "ba_gather"):
            ms, n = ctx.timing_get(k)
            if n:
                res[k] = round(ms / n, 4)
        ctx.timing(False)
        print(json.dumps({"fused": fused, "debug": dbg, "waves": waves, "ms": res}), flush=True)
        dc.free()
ctx.set_option("fused_debug", 0)
