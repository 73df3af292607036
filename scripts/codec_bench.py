#!/usr/bin/env python3
"""Throughput of the codec pass (codec.hip) on C2 / C3
shaped columns: the generator's column, decoded on the GPU, written back by
pyarrow with each codec (default 1 MiB pages), then uploaded with
PQ_EXT_CODECS | PQ_EXT_PAGE_V2: codec kernel time (HIP events), upload wall
time, and the decode checked byte for byte against the uncompressed decode.
usage: codec_bench.py [rows]"""
import hashlib
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import pyarrow.parquet as pq  # noqa: E402

from pqgpu import capi, gen  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
ctx = capi.Context(0)


def to_arrow(h):
    n = h.num_rows
    valid = np.asarray(h.validity)
    bits = np.packbits(valid.astype(bool), bitorder="little")
    return pa.LargeStringArray.from_buffers(n, pa.py_buffer(np.asarray(h.offsets, np.int64).tobytes()),
                                            pa.py_buffer(np.asarray(h.data, np.uint8).tobytes()),
                                            pa.py_buffer(bits.tobytes()), null_count=int(n - valid.sum()))


out = []
for name, cols, layout, seed, use_dict in (("C2", gen.c2_cols(), gen.REF_LAYOUT, 2, True),
                                           ("C3", gen.c3_cols(), gen.REF_LAYOUT, 3, False)):
    f = gen.build(cols, rows, 1, seed=seed, layout=layout)
    dc = ctx.upload(f, [capi.File(f).chunk(0, 0)])
    dc.decode()
    h = dc.to_host()
    dc.free()
    ref = hashlib.sha256(capi.canonical_dump(h)).hexdigest()
    t = pa.table({"s": to_arrow(h)})
    if not cols[0].nullable if hasattr(cols[0], "nullable") else False:
        pass
    for codec in ("snappy", "lz4", "gzip"):
        for ver in ("1.0", "2.0"):
            b = io.BytesIO()
            pq.write_table(t, b, compression=codec.upper() if codec != "lz4" else "LZ4", data_page_version=ver,
                           use_dictionary=use_dict, row_group_size=rows)
            cf = b.getvalue()
            F = capi.File(cf)
            d = F.chunk(0, 0)
            d.ext_flags = capi.EXT_CODECS | capi.EXT_PAGE_V2
            up, ks = [], []
            for _ in range(3):
                ctx.timing(True)
                ctx.timing_reset()
                t0 = time.perf_counter()
                x = ctx.upload(cf, [d])
                up.append(time.perf_counter() - t0)
                ctx.sync()
                ks.append(ctx.timing_get("codec")[0])
                ctx.timing(False)
                if _ < 2:
                    x.free()
            x.decode()
            ok = hashlib.sha256(capi.canonical_dump(x.to_host())).hexdigest() == ref
            ub = x.payload_bytes
            npg = x.num_pages
            x.free()
            kms = sorted(ks)[1]
            r = {"col": name, "codec": codec, "version": ver, "rows": rows, "pages": npg, "file_bytes": len(cf),
                 "uncompressed_payload": ub, "codec_kernel_ms": kms,
                 "codec_GBs_out": ub / (kms * 1e-3) / 1e9 if kms else None,
                 "upload_ms": sorted(up)[1] * 1e3, "validated": ok}
            print(json.dumps(r), flush=True)
            out.append(r)
ctx.close()
