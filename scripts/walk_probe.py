#!/usr/bin/env python3
"""Device page walk (pq_build_page_table_device) vs the host walk
(pq_build_page_table) on the C2 and C3 10M-row chunks: kernel time of the
walk launches (HIP events), wall time of the call, host walk time."""
import json
import sys
import time

sys.path[:0] = ["/root/repo", "/root/repo/duckdb-parquet-parser_amd"]
from pqgpu import capi, gen  # noqa: E402

ctx = capi.Context(0)
for name, cols, seed in (("c2", gen.c2_cols(), gen.CONFIG_SEEDS["C2"]), ("c3", gen.c3_cols(), gen.CONFIG_SEEDS["C3"])):
    f = gen.build(cols, 10_000_000, 1, seed=seed)
    ch = capi.File(f).chunk(0, 0)
    dev = ctx.device_buffer(f)
    t0 = time.perf_counter()
    rc_h, _, host = capi.build_page_table(f, ch)
    th = time.perf_counter() - t0
    out = {"chunk": name, "pages": len(host)}
    for seg in (2048, 8192, 32768):
        ctx.build_page_table_device(dev.data_ptr(), len(f), 0, ch, seg_bytes=seg)  # warm-up
        ctx.timing(True)
        ctx.timing_reset()
        walls = []
        for _ in range(5):
            t0 = time.perf_counter()
            rc, pages = ctx.build_page_table_device(dev.data_ptr(), len(f), 0, ch, seg_bytes=seg)
            walls.append(time.perf_counter() - t0)
        ms, n = ctx.timing_get("walk")
        ctx.timing(False)
        out[f"seg{seg}"] = {"rc": rc, "same": rc == 0 and len(pages) == len(host), "kernel_ms": round(ms / max(n, 1), 4),
                            "call_ms": round(sorted(walls)[2] * 1e3, 3)}
    out["host_walk_ms_python_call"] = round(th * 1e3, 2)
    print(json.dumps(out), flush=True)
