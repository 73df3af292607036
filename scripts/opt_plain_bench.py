#!/usr/bin/env python3
"""OPTIONAL PLAIN BYTE_ARRAY (C3's strings with 5 % NULLs: the shape pyarrow
writes by default) in both layouts: decode time on the default path (levels
-> value sections on the PLAIN kernels), then on the general path (option
plain_fused=0: the fused / generic BYTE_ARRAY kernels), the two outputs
compared byte for byte.  usage: opt_plain_bench.py [rows]"""
import json
import sys
import time
sys.path[:0] = ["/root/repo", "/root/repo/duckdb-parquet-parser_amd"]
from pqgpu import capi, gen  # noqa: E402
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
ctx = capi.Context(0)
cols = [gen.Col("c", gen.COMMENT, gen.BYTE_ARRAY, optional=True, null_frac=0.05, len_min=10, len_max=44)]
KERN = ("ba_fused", "ba_rows", "scan", "ba_gather", "plain_ba", "plain_spec", "fixed_plain", "plain_opt")


def run(f, F):
    dc = ctx.upload(f, [F.chunk(0, 0)])
    dc.decode()
    ctx.sync()
    ctx.timing(True)
    ctx.timing_reset()
    t0 = time.perf_counter()
    for _ in range(5):
        dc.decode_async()
    ctx.sync()
    ms = (time.perf_counter() - t0) * 1e3 / 5
    km = {k: round(ctx.timing_get(k)[0] / 5, 4) for k in KERN if ctx.timing_get(k)[1]}
    ctx.timing(False)
    dump = capi.canonical_dump(dc.to_host())
    pages = dc.num_pages
    dc.free()
    return ms, km, dump, pages


for name, layout in (("ref", gen.REF_LAYOUT), ("arrow", gen.ARROW_LAYOUT)):
    f = gen.build(cols, rows, 1, seed=3, layout=layout)
    F = capi.File(f)
    ms, km, dump, pages = run(f, F)
    ctx.set_option("plain_fused", 0)
    ms_g, km_g, dump_g, _ = run(f, F)
    ctx.set_option("plain_fused", 1)
    print(json.dumps({"layout": name, "pages": pages, "ms_per_decode": round(ms, 4),
                      "Gvalues_s": round(rows / ms / 1e6, 2), "kernels_ms": km,
                      "general_path_ms": round(ms_g, 4), "general_kernels_ms": km_g,
                      "same_as_general_path": dump == dump_g}), flush=True)
