"""Pinned host <-> device copy rates on one GPU (torch, 256 MB and 1 GB), the
ceiling of bench.py's host_pipeline leg."""
import json
import time

import torch

for mb in (64, 256, 1024):
    n = mb << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    for direction in ("h2d", "d2h"):
        for _ in range(2):
            (d.copy_(h, non_blocking=True) if direction == "h2d" else h.copy_(d, non_blocking=True))
        torch.cuda.synchronize()
        t = time.perf_counter()
        reps = 5
        for _ in range(reps):
            (d.copy_(h, non_blocking=True) if direction == "h2d" else h.copy_(d, non_blocking=True))
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / reps
        print(json.dumps({"mb": mb, "dir": direction, "GBps": n / dt / 1e9}), flush=True)
