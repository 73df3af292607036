#!/usr/bin/env python3
"""k_pipe_big phase ablation on the C2 arrow layout (500 pages of 20,000 rows):
option fused_debug bits cut the kernel after staging (0x10000), the header
parse (0x20000), the jump table (4096), the chain walk (8192), the exact
records (16384) and the def levels (32768).  Outputs are not valid under the
ablation.  usage: pipe_big_ablate.py [rows]"""
import json
import sys
sys.path[:0] = ["/root/repo", "/root/repo/duckdb-parquet-parser_amd"]
from pqgpu import capi, gen  # noqa: E402
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
ctx = capi.Context(0)
f = gen.build(gen.c2_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C2"], layout=gen.ARROW_LAYOUT)
F = capi.File(f)
dc = ctx.upload(f, [F.chunk(0, 0)])
for dbg in (0, 0x10000, 0x20000, 4096, 8192, 16384, 32768, 0):
    ctx.set_option("fused_debug", dbg)
    for _ in range(3):
        dc.decode_async()
    ctx.sync()
    ctx.timing(True)
    ctx.timing_reset()
    for _ in range(10):
        dc.decode_async()
    ctx.sync()
    ms, n = ctx.timing_get("pipe_big")
    ctx.timing(False)
    print(json.dumps({"dbg": hex(dbg), "pipe_big_ms": round(ms / max(n, 1), 4)}), flush=True)
