#!/usr/bin/env python3
"""Ablation timings of the BYTE_ARRAY dictionary kernels (C2 shape) on one GPU.

Paths: pipe (dict_pipe.hip), batch (dict_batch.hip), fused (dict_fused.hip),
generic (decode.hip).
fused_debug bits (timing only; the output is not valid with bits set):
  1 = skip the decoupled look-back (fake page bases)
  2 = skip the characters
  4 = skip the offsets stores
  8/16/32 = dict_fused.hip writer internals (see the kernel)
  4096/8192/16384/32768 = k_pipe_big stops after the jump table / chain walk /
      exact records / def levels (`ablate.py arrow big`)
Prints one JSON line per variant with per-kernel average milliseconds, then
per-phase shader-clock cycles (option fused_prof) for the batch and fused
kernels.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-parquet-parser_amd")]
from pqgpu import capi, gen  # noqa: E402

KERNELS = ("dict_index", "pipe_runs", "pipe_big", "pipe_count", "pipe_codes", "pipe_write", "ba_batch", "ba_fused", "ba_rows",
           "scan", "ba_gather")
BATCH_PHASES = ("p_waitbuf", "p_stage", "p_walk", "p_lookback", "batches",
                "w_wait", "w_runs", "w_rows", "w_chars", "pages", "p_defwalk")

rows = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10_000_000
layout = gen.ARROW_LAYOUT if "arrow" in sys.argv else gen.REF_LAYOUT
f = gen.build(gen.c2_cols(), rows, 1, seed=gen.CONFIG_SEEDS["C2"], layout=layout)
F = capi.File(f)
chunks = [F.chunk(0, 0)]
ctx = capi.Context(0)


def setp(path, dbg=0, waves=0, bbytes=12288, claim=1, rp=32, wmode=0):
    ctx.set_option("pipe_run_pages", rp)
    ctx.set_option("dict_pipe", int(path == "pipe"))
    ctx.set_option("fused_claim", claim)
    ctx.set_option("fused_ba", int(path != "generic"))
    ctx.set_option("batch", int(path == "batch"))
    ctx.set_option("fused_debug", dbg)
    ctx.set_option("fused_waves", waves)
    ctx.set_option("batch_bytes", bbytes)


variants = [("pipe", 0, 0, 12288, 1), ("pipe", 2, 0, 12288, 1), ("pipe", 4, 0, 12288, 1),
            ("pipe", 6, 0, 12288, 1), ("fused", 0, 0, 12288, 1)]
if "codes" in sys.argv:
    variants = [("pipe", d, 0, 12288, 1) for d in (0, 512, 1024)]
if "write" in sys.argv:
    variants = [("pipe", d, 0, 12288, 1, 32, wm) for wm in (0,) for d in (0, 2, 4, 6)]
if "runpages" in sys.argv:
    variants = [("pipe", 0, 0, 12288, 1, rp) for rp in (32, 16, 8, 4)]
if "big" in sys.argv:  # k_pipe_big phases (arrow layout): jump table, walk, records, def levels, all
    variants = [("pipe", d, 0, 12288, 1) for d in (4096, 8192, 16384, 32768, 0)]
if "batch" in sys.argv:
    variants += [("batch", 0, 0, 12288, 1), ("batch", 1, 0, 12288, 1), ("batch", 3, 0, 12288, 1)]
for v in variants:
    path, dbg, waves, bb, claim = v[:5]
    rp = v[5] if len(v) > 5 else 32
    wm = v[6] if len(v) > 6 else 0
    setp(path, 0, waves, bb, claim, rp, wm)
    dc = ctx.upload(f, chunks)
    dc.decode_async()  # valid intermediate buffers before any ablation bit is set
    ctx.sync()
    ctx.set_option("fused_debug", dbg)
    dc.decode_async()
    ctx.sync()
    ctx.timing(True)
    ctx.timing_reset()
    for _ in range(10):
        dc.decode_async()
    ctx.sync()
    res = {}
    for k in KERNELS:
        ms, n = ctx.timing_get(k)
        if n:
            res[k] = round(ms / n, 4)
    ctx.timing(False)
    print(json.dumps({"path": path, "debug": dbg, "write_mode": wm, "waves": waves, "batch_bytes": bb, "claim": claim, "run_pages": rp,
                      "ms": res}),
          flush=True)
    dc.free()

ctx.set_option("fused_prof", 1)
for path in (("batch", "fused") if "prof" in sys.argv else ()):
    setp(path)
    dc = ctx.upload(f, chunks)
    dc.decode_async()
    ctx.sync()
    ctx.fused_prof_read()
    for _ in range(5):
        dc.decode_async()
    ctx.sync()
    raw = ctx.fused_prof_read(raw=True)
    if path == "batch":
        pr = dict(zip(BATCH_PHASES, raw))
        nb, npg = max(pr["batches"], 1), max(pr["pages"], 1)
        out = {k: round(v / nb) for k, v in pr.items() if k.startswith("p_")}
        out.update({k: round(v / npg) for k, v in pr.items() if k.startswith("w_")})
        print(json.dumps({"path": path, "cycles (producer per batch, writer per page)": out,
                          "batches": nb, "pages": npg}), flush=True)
    else:
        pr = dict(zip(capi.Context.PROF_PHASES, raw))
        npg = max(pr.get("pages", 1), 1)
        print(json.dumps({"path": path, "cycles_per_page": {k: round(v / npg) for k, v in pr.items()
                                                           if k not in ("pages", "w_pages")}}), flush=True)
    dc.free()
ctx.set_option("fused_prof", 0)
setp("batch")
