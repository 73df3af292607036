#!/usr/bin/env python3
"""HBM write-rate reference points on one GPU: torch fill_ (a streaming store
kernel) and hipMemsetAsync-backed zero_ over buffers the size of the C2
pipe_write output (218 MB characters + 80 MB offsets)."""
import time
import torch

dev = torch.device("cuda:0")
for mb in (80, 218, 300, 1024):
    x = torch.empty(mb * 1000 * 1000, dtype=torch.uint8, device=dev)
    for name, fn in (("fill_", lambda: x.fill_(7)), ("zero_", lambda: x.zero_())):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        n = 20
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / n
        print(f"{name} {mb} MB: {ms * 1e3:.1f} us  {mb * 1e6 / (ms * 1e-3) / 1e12:.2f} TB/s", flush=True)
    del x
