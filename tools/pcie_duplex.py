"""PCIe duplex probe: H2D and D2H of pinned host memory, alone and concurrently (two HIP streams)."""
import json
import time

import torch

N = 4 << 30
h_src = torch.empty(N, dtype=torch.uint8, pin_memory=True)
h_dst = torch.empty(N, dtype=torch.uint8, pin_memory=True)
d_a = torch.empty(N, dtype=torch.uint8, device="cuda")
d_b = torch.empty(N, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def run(h2d, d2h, reps=3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        if h2d:
            with torch.cuda.stream(s1):
                d_a.copy_(h_src, non_blocking=True)
        if d2h:
            with torch.cuda.stream(s2):
                h_dst.copy_(d_b, non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return round((N * (int(h2d) + int(d2h))) / dt / 1e9, 1)


run(True, True, 1)
print(json.dumps({"h2d_gbps": run(True, False), "d2h_gbps": run(False, True), "both_aggregate_gbps": run(True, True)}))
