import sys; sys.path[:0]=['/root/repo','/root/repo/duckdb-parquet-parser_amd','/root/repo/tests']
from pqgpu import gen, capi
from util import file_chunks
ctx = capi.Context(0)
for rows in (20000, 40000, 100000):
    f = gen.build([gen.c4_cols()[7]], rows, 1, seed=4, layout=gen.ARROW_LAYOUT)
    ch = file_chunks(f, 0)
    dc = ctx.upload(f, ch)
    dc.decode()
    ctx.timing(True); ctx.timing_reset(); dc.decode_async(); ctx.sync()
    print(rows, dc.num_pages, "spec", ctx.timing_get("plain_spec"), "generic", ctx.timing_get("ba_rows"))
    ctx.timing(False); dc.decode_check(); dc.free()
