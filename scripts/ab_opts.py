#!/usr/bin/env python3
"""A/B of context options on one column: per-kernel times (HIP events), the
step's wall time without timers, and a byte-for-byte check of every variant's
output against the first variant's.
usage: ab_opts.py CONFIG[:col] [rows] VARIANT...
  VARIANT = "-" (defaults) or "key=value,key=value" (options set before upload)
  e.g. ab_opts.py C2 10000000 - big_all=1"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# AB_PKG: a directory holding another build's pqgpu package (A/B of compile-time constants)
sys.path[:0] = [ROOT, os.environ.get("AB_PKG") or os.path.join(ROOT, "duckdb-parquet-parser_amd")]
import numpy as np  # noqa: E402
from pqgpu import capi, gen  # noqa: E402

CONFIGS = {"C2": (gen.c2_cols, gen.REF_LAYOUT, 2), "C2a": (gen.c2_cols, gen.ARROW_LAYOUT, 2),
           "C3": (gen.c3_cols, gen.REF_LAYOUT, 3), "C4": (gen.c4_cols, gen.ARROW_LAYOUT, 4),
           # bench.py's wide_dict leg: the C2 shape with a 100,000-entry dictionary
           "W": (lambda: [gen.Col("s", gen.DICT_STRINGS, gen.BYTE_ARRAY, optional=True, null_frac=0.05,
                                  dict_size=100_000, len_min=4, len_max=9, max_run=16)], gen.ARROW_LAYOUT, 2)}
# library defaults of the options the variants may set (restored after each)
DEFAULTS = {"pipe_run_pages": 32, "pipe_run_dict": 1, "regex_index": 1, "zflip": 1, "write_waves": 10, "dict_pipe": 1, "plain_ba": 1,
            "fused_ba": 1, "fixed_plain": 1, "fixed_fused": 0, "big_all": 0, "fused_debug": 0, "plain_fused": 1, "regex_win": 8192,
            "raw_upload": 1, "write_bpc": 0, "wide_rows": 1, "gather_rows": 1, "levels_small": 1, "pipe_wide": 1}
KERNELS = ("dict_index", "dict_entries", "pipe_runs", "pipe_big", "wide_chars", "plain_spec", "pipe_count", "pipe_codes",
           "pipe_write", "ba_fused", "ba_rows", "scan", "ba_gather", "fixed", "fixed_plain", "plain_ba", "plain_opt")

cfg, _, colname = sys.argv[1].partition(":")
rows = int(sys.argv[2])
variants = sys.argv[3:] or ["-"]
mk, layout, seed = CONFIGS[cfg]
cols = mk()
ci = next((i for i, c in enumerate(cols) if c.name == colname), 0) if colname else 0
f = gen.build(cols, rows, 1, seed=seed, layout=layout)
F = capi.File(f)
# one context (several contexts share the process's hardware queues and
# disturb each other's wall clock); each round uploads the column again under
# every variant's options, in rotating order; medians are reported
ctx = capi.Context(0)
parsed = []
for v in variants:
    parsed.append({} if v == "-" else {k: int(x) for k, x in (kv.split("=") for kv in v.split(","))})
defaults = {}
res = [{"wall": [], "ms": [], "same": None} for _ in variants]
base = None
for rnd in range(3):
    order = list(range(len(variants)))
    order = order[rnd % len(order):] + order[:rnd % len(order)]
    for i in order:
        for k, x in parsed[i].items():
            ctx.set_option(k, x)
        dc = ctx.upload(f, [F.chunk(0, ci)])
        try:
            dc.decode()
        except capi.PqError as e:  # timing probes (debug bits) may leave invalid output
            print(f"variant {variants[i]}: {e}", file=sys.stderr)
        if rnd == 0:
            h = dc.to_host()
            if i == 0:
                base = h
        for _ in range(20):
            dc.decode_async()
        ctx.sync()
        steps = 50
        t0 = time.perf_counter()
        for _ in range(steps):
            dc.decode_async()
        ctx.sync()
        res[i]["wall"].append((time.perf_counter() - t0) / steps * 1e3)
        ctx.timing(True)
        ctx.timing_reset()
        for _ in range(10):
            dc.decode_async()
        ctx.sync()
        res[i]["ms"].append({k: ctx.timing_get(k)[0] / 10 for k in KERNELS if ctx.timing_get(k)[1]})
        ctx.timing(False)
        if rnd == 0 and i != 0:
            res[i]["h"] = dc.to_host()
        dc.free()
        for k in parsed[i]:  # back to the defaults of the library
            ctx.set_option(k, DEFAULTS.get(k, 0))
for i, v in enumerate(variants):
    same = None
    if i and base is not None and "h" in res[i]:
        h = res[i]["h"]
        same = bool(np.array_equal(h.validity, base.validity) and np.array_equal(h.data, base.data) and
                    (h.offsets is None or np.array_equal(h.offsets, base.offsets)))
    walls = sorted(res[i]["wall"])
    wall = walls[len(walls) // 2]
    ks = res[i]["ms"][0].keys()
    ms = {k: round(sorted(r.get(k, 0.0) for r in res[i]["ms"])[1], 4) for k in ks}
    print(json.dumps({"variant": v, "same_as_first": same, "wall_ms": round(wall, 4),
                      "Gvalues_s": round(rows / wall / 1e6, 2), "ms": ms}), flush=True)
