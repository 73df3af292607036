#!/usr/bin/env python3
"""Upload (host walk + plan + pinned H2D) phase timings of the C3 10M-row
chunk for a few staging-ring shapes (options stage_bufs / stage_piece_kb)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
from pqgpu import capi, gen  # noqa: E402

f = gen.build(gen.c3_cols(), 10_000_000, 1, seed=3)
ch = capi.File(f).chunk(0, 0)
ctx = capi.Context(0)
for streams, bufs, kb in [(1, 6, 8192), (2, 6, 8192), (2, 8, 4096), (2, 8, 16384), (2, 12, 4096), (1, 8, 16384)]:
    ctx.set_option("stage_streams", streams)
    ctx.set_option("stage_bufs", bufs)
    ctx.set_option("stage_piece_kb", kb)
    x = ctx.upload(f, [ch])
    x.free()
    ctx.timing(True)
    ctx.timing_reset()
    ts = []
    for _ in range(4):
        t0 = time.perf_counter()
        x = ctx.upload(f, [ch])
        ts.append(time.perf_counter() - t0)
        x.free()
    ctx.timing(False)
    ph = {k: round(ctx.timing_get(k)[0] / 4, 3) for k in ("up_walk", "up_plan", "up_alloc", "up_h2d", "up_fill", "up_wait")}
    print(f"streams {streams} bufs {bufs:2d} piece {kb:6d} KiB: upload {min(ts) * 1e3:.2f} ms  {ph}", flush=True)
