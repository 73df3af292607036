#!/usr/bin/env python3
"""Achievable HBM rates on this box for the writer's roofline context: a
300 MB fill (write only) and a 300 MB device copy (read + write), timed with
HIP events over 20 repetitions (torch; the device buffers only)."""
import json

import torch

n = 300 * 1000 * 1000
a = torch.empty(n, dtype=torch.uint8, device="cuda")
b = torch.empty(n, dtype=torch.uint8, device="cuda")
out = {}
for name, fn, bytes_moved in (("fill", lambda: a.fill_(1), n), ("copy", lambda: b.copy_(a), 2 * n)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    out[name] = {"ms": round(ms, 4), "GB_s": round(bytes_moved / ms / 1e6, 1)}
print(json.dumps(out))
