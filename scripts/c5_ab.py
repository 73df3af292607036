#!/usr/bin/env python3
"""C5 decode wall time per row group under context options and stream counts:
N row groups of the C5 column (arrow layout), alternated over S contexts,
every variant's output checked against the first variant's.
usage: c5_ab.py [rgs] VARIANT...   VARIANT = "S" or "S:key=value+key=value"
(options are set on every context before upload)"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.environ.get("AB_PKG") or os.path.join(ROOT, "duckdb-parquet-parser_amd")]
from pqgpu import capi, gen  # noqa: E402

rgs = int(sys.argv[1]) if len(sys.argv) > 1 else 6
variants = sys.argv[2:] or ["2", "2:write_bpc=1", "3"]
f = gen.build(gen.c2_cols(), 10_000_000, rgs, seed=gen.CONFIG_SEEDS["C5"], layout=gen.ARROW_LAYOUT)
F = capi.File(f)
ctxs = [capi.Context(0) for _ in range(4)]
ref = None
for v in variants:
    S, _, o = v.partition(":")
    S = int(S)
    opts = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in o.split("+") if kv)
    for c in ctxs[:S]:
        for k, x in opts.items():
            c.set_option(k, x)
    dcs = [ctxs[i % S].upload(f, [F.chunk(i, 0)]) for i in range(rgs)]
    h = hashlib.sha256()
    for d in dcs:
        d.decode()
        h.update(capi.canonical_dump(d.to_host()))
    same = ref is None or h.hexdigest() == ref
    ref = ref or h.hexdigest()
    walls = []
    for _ in range(5):
        for d in dcs:
            d.decode_async()
        for c in ctxs[:S]:
            c.sync()
        t0 = time.perf_counter()
        for _ in range(5):
            for d in dcs:
                d.decode_async()
        for c in ctxs[:S]:
            c.sync()
        walls.append((time.perf_counter() - t0) / 5 / rgs * 1e3)
    walls.sort()
    print(json.dumps({"variant": v, "same": same, "ms_per_rg": round(walls[2], 4),
                      "Gvalues_s": round(10.0 / walls[2], 2)}), flush=True)
    for d in dcs:
        d.free()
    for c in ctxs[:S]:
        for k in opts:
            c.set_option(k, {"write_bpc": 0, "write_waves": 10}.get(k, 0))
