"""Probe: does an H2D DMA from pinned memory slow concurrent CPU memcpys into pinned memory?

The NetMerger's fetch writes partitions into pinned arenas with many threads while the early stager
copies landed bytes to HBM. This measures the CPU copy rate (pageable -> pinned, like a loopback fetch)
  alone, next to an H2D of an unrelated pinned buffer, and chasing its own writes (each 8 MiB piece
  copied to the device as soon as it is written)."""
import json
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

GB = 2 << 30
PIECE = 8 << 20
THREADS = 16
src = np.random.randint(0, 255, size=GB, dtype=np.uint8)
dst_t = torch.empty(GB, dtype=torch.uint8, pin_memory=True)
dst = dst_t.numpy()
other = torch.empty(GB, dtype=torch.uint8, pin_memory=True)
dev = torch.empty(GB, dtype=torch.uint8, device="cuda")
dev2 = torch.empty(GB, dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
lock = threading.Lock()


def cpu_copy(chase=False):
    n = GB // PIECE
    per = n // THREADS

    def work(t):
        for i in range(t * per, (t + 1) * per):
            a, b = i * PIECE, (i + 1) * PIECE
            np.copyto(dst[a:b], src[a:b])
            if chase:
                with lock, torch.cuda.stream(s):
                    dev[a:b].copy_(dst_t[a:b], non_blocking=True)

    t0 = time.perf_counter()
    with ThreadPoolExecutor(THREADS) as ex:
        list(ex.map(work, range(THREADS)))
    dt = time.perf_counter() - t0
    s.synchronize()
    return round(GB / dt / 1e9, 1), round((time.perf_counter() - t0) * 1e3, 1)


def background_h2d(stop):
    with torch.cuda.stream(s):
        while not stop.is_set():
            dev2.copy_(other, non_blocking=True)
            s.synchronize()


cpu_copy()
out = {"alone_gbps_ms": cpu_copy()}
stop = threading.Event()
th = threading.Thread(target=background_h2d, args=(stop,))
th.start()
time.sleep(0.05)
out["beside_unrelated_h2d_gbps_ms"] = cpu_copy()
stop.set()
th.join()
out["chasing_own_writes_gbps_ms"] = cpu_copy(chase=True)
out["alone_again_gbps_ms"] = cpu_copy()
print(json.dumps(out))
