#!/usr/bin/env python3
"""A/B of the codec pass's options on C3's column as pyarrow writes it
(SNAPPY / LZ4 / LZ4_RAW / ZSTD; 1 MiB pages and 8 KiB pages): the codec
kernel's time (HIP events) per option set, every variant's decode checked
against the uncompressed decode.
usage: codec_ab.py [rows] [opt=val[:reset],...]...  (reset: the value restored
after the variant, default 0)"""
import hashlib
import io
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# AB_PKG: a directory holding another build's pqgpu package (probe builds)
sys.path[:0] = [ROOT, os.environ.get("AB_PKG") or os.path.join(ROOT, "duckdb-parquet-parser_amd")]
import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import pyarrow.parquet as pq  # noqa: E402

from pqgpu import capi, gen  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
variants = sys.argv[2:] or ["-"]
ctx = capi.Context(0)
f = gen.build(gen.c3_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C3"])
dc = ctx.upload(f, [capi.File(f).chunk(0, 0)])
dc.decode()
h = dc.to_host()
dc.free()
ref = hashlib.sha256(capi.canonical_dump(h)).hexdigest()
valid = np.asarray(h.validity)
arr = pa.LargeStringArray.from_buffers(h.num_rows, pa.py_buffer(np.asarray(h.offsets, np.int64).tobytes()),
                                       pa.py_buffer(np.asarray(h.data, np.uint8).tobytes()),
                                       pa.py_buffer(np.packbits(valid.astype(bool), bitorder="little").tobytes()),
                                       null_count=int(h.num_rows - valid.sum()))
del h
for codec, ver, page in (("SNAPPY", "1.0", 1 << 20), ("SNAPPY", "1.0", 8192), ("LZ4", "2.0", 1 << 20),
                         ("ZSTD", "1.0", 1 << 20), ("ZSTD", "1.0", 8192)):
    b = io.BytesIO()
    pq.write_table(pa.table({"s": arr}), b, compression=codec, data_page_version=ver, use_dictionary=False,
                   row_group_size=rows, data_page_size=page)
    cf = b.getvalue()
    d = capi.File(cf).chunk(0, 0)
    d.ext_flags = capi.EXT_CODECS | capi.EXT_PAGE_V2
    for v in variants:
        opts = {} if v == "-" else {k: (x + ":0").split(":")[:2] for k, x in (kv.split("=") for kv in v.split(","))}
        for k, (x, _) in opts.items():
            ctx.set_option(k, int(x))
        ms = []
        for _ in range(3):
            ctx.timing(True)
            ctx.timing_reset()
            x = ctx.upload(cf, [d])
            ctx.sync()
            ms.append(ctx.timing_get("codec")[0])
            ctx.timing(False)
            x.free()
        x = ctx.upload(cf, [d])
        try:
            x.decode()
            ok = hashlib.sha256(capi.canonical_dump(x.to_host())).hexdigest() == ref
        except capi.PqError:  # timing probes leave invalid pages
            ok = False
        ub = x.payload_bytes
        x.free()
        for k, (_, r) in opts.items():
            ctx.set_option(k, int(r))
        m = statistics.median(ms)
        print(json.dumps({"codec": codec, "version": ver, "page": page, "variant": v, "codec_ms": round(m, 3),
                          "GBs_out": round(ub / (m * 1e-3) / 1e9, 2), "validated": ok}), flush=True)
