#!/usr/bin/env python3
"""Run the C2 decode, the C3 regex scan or the C3 PLAIN decode a few times — a
small target for rocprofv3 PMC passes.
usage: kernel_driver.py [decode|regex|plain|optplain|c4|c5|wide] [rows] [reps] [fused_debug]
(c4: env PQ_COLS="3,7" picks the C4 columns; wide: the 100k-entry dictionary)
(env PQ_OPTS="key=value,..." sets further context options)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
from pqgpu import capi, gen  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "decode"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dbg = int(sys.argv[4]) if len(sys.argv) > 4 else 0
ctx = capi.Context(0)
ctx.set_option("fused_debug", dbg)
for kv in filter(None, os.environ.get("PQ_OPTS", "").split(",")):  # e.g. PQ_OPTS=regex_debug=1
    k, v = kv.split("=")
    ctx.set_option(k, int(v))
if what == "decode":
    f = gen.build(gen.c2_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C2"])
    F = capi.File(f)
    dc = ctx.upload(f, [F.chunk(0, 0)])
    for _ in range(reps):
        dc.decode_async()
    ctx.sync()
elif what == "c4":
    cols = gen.c4_cols()
    f = gen.build(cols, rows, 1, seed=gen.CONFIG_SEEDS["C4"], layout=gen.ARROW_LAYOUT)
    F = capi.File(f)
    for ci in [int(x) for x in os.environ.get("PQ_COLS", "3").split(",")]:
        dc = ctx.upload(f, [F.chunk(0, ci)])
        for _ in range(reps):
            dc.decode_async()
        ctx.sync()
        dc.free()
elif what == "optplain":  # C3's strings OPTIONAL, 5 % NULL, arrow 20,000-row pages (bench c3_decode.optional_arrow)
    col = gen.Col("comment", gen.COMMENT, gen.BYTE_ARRAY, optional=True, null_frac=0.05, len_min=10, len_max=44)
    f = gen.build([col], rows, 1, seed=gen.CONFIG_SEEDS["C3"], layout=gen.ARROW_LAYOUT)
    dc = ctx.upload(f, [capi.File(f).chunk(0, 0)])
    for _ in range(reps):
        dc.decode_async()
    ctx.sync()
elif what == "c5":  # C5 arrow row group(s): decode + one-pass filter
    f = gen.build(gen.c2_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C5"], layout=gen.ARROW_LAYOUT)
    dc = ctx.upload(f, [capi.File(f).chunk(0, 0)])
    dc.decode()
    for _ in range(reps):
        dc.decode_async()
    for _ in range(reps):
        dc.decode_regex_async("^qx")
    ctx.sync()
elif what == "wide":
    col = gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=0.05, dict_size=100_000,
                  len_min=4, len_max=9, max_run=16)
    f = gen.build([col], rows, 1, seed=gen.CONFIG_SEEDS["C2"], layout=gen.ARROW_LAYOUT)
    dc = ctx.upload(f, [capi.File(f).chunk(0, 0)])
    for _ in range(reps):
        dc.decode_async()
    ctx.sync()
elif what == "plain":
    f = gen.build(gen.c3_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C3"])
    F = capi.File(f)
    dc = ctx.upload(f, [F.chunk(0, 0)])
    for _ in range(reps):
        dc.decode_async()
    ctx.sync()
else:
    f = gen.build(gen.c3_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C3"])
    F = capi.File(f)
    dc = ctx.upload(f, [F.chunk(0, 0)])
    for _ in range(reps):
        dc.regex_pages("special.*requests", False)
    ctx.sync()
print("done", what, rows, reps)
