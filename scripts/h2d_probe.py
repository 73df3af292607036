#!/usr/bin/env python3
"""Host-to-device floor of the end-to-end numbers: H2D of C3's chunk size
(310 MB) and C2's (7.6 MB) from pinned and from pageable host memory (torch
copies, median of 5).  usage: h2d_probe.py"""
import json
import statistics
import time

import torch

dev = torch.device("cuda:0")
out = {}
for name, n in (("c3", 310_581_303), ("c2", 7_572_276)):
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    for kind in ("pinned", "pageable"):
        h = torch.empty(n, dtype=torch.uint8, pin_memory=(kind == "pinned"))
        h.fill_(1)
        ts = []
        for _ in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            d.copy_(h, non_blocking=(kind == "pinned"))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ms = statistics.median(ts[1:]) * 1e3
        out[f"{name}_{kind}"] = {"bytes": n, "ms": round(ms, 4), "GBs": round(n / ms / 1e6, 2)}
print(json.dumps(out))
