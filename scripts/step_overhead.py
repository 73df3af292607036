#!/usr/bin/env python3
"""C2 decode step wall time with and without the per-kernel HIP-event
timers (ctx.timing) inside the timed loop, with and without the
captured HIP graph.  usage: step_overhead.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
from pqgpu import capi, gen  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
ctx = capi.Context(0)
f = gen.build(gen.c2_cols(), 10_000_000, 1, seed=gen.CONFIG_SEEDS["C2"])
F = capi.File(f)
dc = ctx.upload(f, [F.chunk(0, 0)])
dc.decode()
for graph, timing in ((1, False), (0, False), (1, True), (1, False)):
    ctx.set_option("graph", graph)
    ctx.timing(timing)
    for _ in range(5):
        dc.decode_async()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        dc.decode_async()
    t1 = time.perf_counter()
    ctx.sync()
    t2 = time.perf_counter()
    ctx.timing(False)
    print(f"graph={graph} timing={timing}: {(t2 - t0) / steps * 1e3:.4f} ms/step wall, host enqueue {(t1 - t0) / steps * 1e3:.4f} ms/step")
