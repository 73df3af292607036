#!/usr/bin/env python3
"""Upload phases of a pyarrow-written C3 file (SNAPPY, V1 pages, 1 MiB
pages): host walk / plan / allocation / H2D, the codec pass and the first
decode, to see where a compressed upload spends its time.
usage: ext_upload_phases.py [rows] [codec]"""
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
import pyarrow as pa  # noqa: E402
import pyarrow.parquet as pq  # noqa: E402
from pqgpu import capi, gen  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
codec = sys.argv[2] if len(sys.argv) > 2 else "SNAPPY"
ctx = capi.Context(0)
f = gen.build(gen.c3_cols(), rows, 1, seed=3)
dc = ctx.upload(f, [capi.File(f).chunk(0, 0)])
dc.decode()
h = dc.to_host()
dc.free()
import numpy as np  # noqa: E402
arr = pa.LargeStringArray.from_buffers(h.num_rows, pa.py_buffer(np.asarray(h.offsets, np.int64).tobytes()),
                                       pa.py_buffer(np.asarray(h.data, np.uint8).tobytes()))
b = io.BytesIO()
pq.write_table(pa.table({"s": arr}), b, compression=codec, use_dictionary=False, row_group_size=rows)
cf = b.getvalue()
d = capi.File(cf).chunk(0, 0)
d.ext_flags = capi.EXT_CODECS | capi.EXT_PAGE_V2
KEYS = ("up_walk", "up_plan", "up_alloc", "up_h2d", "up_fill", "up_wait", "codec", "relayout")
for i in range(3):
    ctx.timing(True)
    ctx.timing_reset()
    t0 = time.perf_counter()
    x = ctx.upload(cf, [d])
    t1 = time.perf_counter()
    x.decode()
    t2 = time.perf_counter()
    ph = {k: round(ctx.timing_get(k)[0], 3) for k in KEYS if ctx.timing_get(k)[1]}
    ctx.timing(False)
    print(json.dumps({"file_MB": round(len(cf) / 1e6, 1), "pages": x.num_pages, "upload_ms": round((t1 - t0) * 1e3, 2),
                      "first_decode_ms": round((t2 - t1) * 1e3, 2), "phases_ms": ph}), flush=True)
    x.free()
