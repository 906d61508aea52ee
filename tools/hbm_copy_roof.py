#!/usr/bin/env python3
"""HBM roof for the merge: device-to-device copy of an 8.1 GB buffer (one K-way round's records) with
hipMemcpy (blit kernel) and with torch's elementwise copy; reports read+write TB/s (each byte read once
and written once, the K-way kernel's own HBM traffic per record)."""
import json
import time

import torch


def bench(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


n = 8_125_000_000
a = torch.empty(n, dtype=torch.uint8, device="cuda")
b = torch.empty_like(a)
a.fill_(7)
out = {}
t = bench(lambda: b.copy_(a))
out["torch_copy_ms"] = round(t * 1e3, 3)
out["torch_copy_rw_tbps"] = round(2 * n / t / 1e12, 3)
a64, b64 = a.view(torch.int64), b.view(torch.int64)
t = bench(lambda: torch.add(a64, 1, out=b64))
out["add1_i64_ms"] = round(t * 1e3, 3)
out["add1_i64_rw_tbps"] = round(2 * n / t / 1e12, 3)
print(json.dumps(out), flush=True)
