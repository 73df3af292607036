#!/usr/bin/env python3
"""Timing probe: one C2 column decoded as R page-range sub-chunks spread over
S contexts (HIP streams), so one range's latency-bound front kernels can run
beside another range's bandwidth-bound k_pipe_write.  Prints the wall time
per whole-column decode for each (R, S, options) and checks every variant's
concatenated output against the unsplit decode.
usage: overlap_probe.py [rows] [R:S[:opts] ...]   (opts: key=value+key=value)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
import numpy as np  # noqa: E402
from pqgpu import capi, gen, shard  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
variants = sys.argv[2:] or ["1:1", "2:2", "4:2", "8:2"]
f = gen.build(gen.c2_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C2"])
F = capi.File(f)
ch = F.chunk(0, 0)
rc, msg, table = capi.build_page_table(f, ch)
assert rc == 0, msg
ctxs = [capi.Context(0) for _ in range(int(os.environ.get("NCTX", "2")))]

ref = ctxs[0].upload(f, [ch])
ref.decode()
base = ref.to_host()
ref.free()

for v in variants:
    parts = v.split(":")
    R, S = int(parts[0]), int(parts[1])
    opts = {}
    if len(parts) > 2:
        for kv in parts[2].split("+"):
            k, x = kv.split("=")
            opts[k] = int(x)
    for c in ctxs[:S]:
        for k, x in opts.items():
            c.set_option(k, x)
    ranges = shard.data_page_ranges(table, R)
    dcs = [ctxs[i % S].upload_range(f, ch, table, b, e) for i, (b, e) in enumerate(ranges)]
    for d in dcs:
        d.decode()
    # output check: concatenation of the ranges == the unsplit decode (offsets rebased)
    ok = True
    off = 0
    char0 = 0
    for d in dcs:
        h = d.to_host()
        n = h.num_rows if hasattr(h, "num_rows") else len(h.offsets) - 1
        if h.offsets is not None:
            ok &= bool(np.array_equal(h.offsets - h.offsets[0] + base.offsets[off], base.offsets[off:off + n + 1]))
            ok &= bytes(h.data[:int(h.offsets[-1])]) == bytes(base.data[base.offsets[off]:base.offsets[off + n]])
        off += n
    walls = []
    for rnd in range(5):
        for _ in range(5):
            for d in dcs:
                d.decode_async()
        for c in ctxs[:S]:
            c.sync()
        steps = 20
        t0 = time.perf_counter()
        for _ in range(steps):
            for d in dcs:
                d.decode_async()
        for c in ctxs[:S]:
            c.sync()
        walls.append((time.perf_counter() - t0) / steps * 1e3)
    walls.sort()
    print(json.dumps({"R": R, "S": S, "opts": opts, "same": ok, "wall_ms": round(walls[2], 4),
                      "Gvalues_s": round(rows / walls[2] / 1e6, 2)}), flush=True)
    for d in dcs:
        d.free()
    for c in ctxs[:S]:
        for k in opts:
            c.set_option(k, {"dict_pipe": 1, "write_waves": 10}.get(k, 0))
