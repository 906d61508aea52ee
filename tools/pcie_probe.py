#!/usr/bin/env python3
"""Host<->device copy ceiling on this box: the roof the headline bench is measured against.

bench.py is bound by D2H (every merged byte reaches the host reducer through dataFromUda), so its
GB/s is only meaningful next to what the PCIe link delivers here. This probe times pinned
hipMemcpyAsync copies (through torch: copy_ with non_blocking=True) for several piece sizes and
stream counts, D2H, H2D and both directions at once, and prints one JSON object.

    python tools/pcie_probe.py [--total-gb 16] [--out gpurun_out/pcie_probe.json]
"""
from __future__ import annotations

import argparse
import json
import time

import torch


def timed_copies(dst, src, pieces, streams, reps):
    """Copy src->dst piece by piece, round-robin over streams; returns GB/s."""
    n = src.numel()
    step = n // pieces
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for i in range(pieces):
            with torch.cuda.stream(streams[i % len(streams)]):
                dst[i * step:(i + 1) * step].copy_(src[i * step:(i + 1) * step], non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return reps * pieces * step / dt / 1e9


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--total-gb", type=float, default=8.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    n = int(a.total_gb * 1e9) // (256 << 20) * (256 << 20)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    dev2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    host2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    dev.random_(0, 255)
    host2.fill_(7)
    ss = [torch.cuda.Stream() for _ in range(4)]
    res = {"device": torch.cuda.get_device_name(0), "bytes": n, "d2h": {}, "h2d": {}, "bidir": {}}
    for piece_mb in (1, 16, 64, 256):
        pieces = n // (piece_mb << 20)
        for k in (1, 2, 4):
            timed_copies(host, dev, pieces, ss[:k], 1)  # warm
            res["d2h"][f"{piece_mb}MiB_x{k}"] = round(timed_copies(host, dev, pieces, ss[:k], a.reps), 2)
            res["h2d"][f"{piece_mb}MiB_x{k}"] = round(timed_copies(dev2, host2, pieces, ss[:k], a.reps), 2)
    # both directions at once: D2H on stream 0, H2D on stream 1
    pieces = n // (64 << 20)
    step = n // pieces
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        for i in range(pieces):
            with torch.cuda.stream(ss[0]):
                host[i * step:(i + 1) * step].copy_(dev[i * step:(i + 1) * step], non_blocking=True)
            with torch.cuda.stream(ss[1]):
                dev2[i * step:(i + 1) * step].copy_(host2[i * step:(i + 1) * step], non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res["bidir"]["64MiB_each_way_GBps"] = round(a.reps * n / dt / 1e9, 2)
    res["d2h_peak"] = max(res["d2h"].values())
    res["h2d_peak"] = max(res["h2d"].values())
    s = json.dumps(res)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
