"""Probe 2: the NetMerger fetch pattern. 8 writer threads fill 64 partitions of a pinned arena in
1 MiB chunks (partitions interleaved, like concurrent drains), while a stager thread copies each
partition's landed prefix to the device every STEP bytes (hipMemcpyAsync via torch, on its own
stream). Prints the writers' time with and without the stager."""
import json
import queue
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

PARTS, PART = 64, 32 << 20
CHUNK = 1 << 20
STEP = int(sys.argv[1]) if len(sys.argv) > 1 else (8 << 20)
src = np.random.randint(0, 255, size=PART, dtype=np.uint8)
arena_t = torch.empty(PARTS * PART, dtype=torch.uint8, pin_memory=True)
arena = arena_t.numpy()
dev = torch.empty(PARTS * PART, dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()


def run(stage: bool):
    q: queue.Queue = queue.Queue()
    landed = [0] * PARTS
    reported = [0] * PARTS
    lock = threading.Lock()

    def stager():
        with torch.cuda.stream(s):
            while True:
                item = q.get()
                if item is None:
                    return
                a, b = item
                dev[a:b].copy_(arena_t[a:b], non_blocking=True)

    th = threading.Thread(target=stager)
    th.start()
    order = [(p, c) for c in range(PART // CHUNK) for p in range(PARTS)]  # interleaved

    def work(k):
        for i in range(k, len(order), 8):
            p, c = order[i]
            off = p * PART + c * CHUNK
            np.copyto(arena[off:off + CHUNK], src[c * CHUNK:(c + 1) * CHUNK])
            if stage:
                with lock:
                    landed[p] += CHUNK
                    if landed[p] - reported[p] >= STEP or landed[p] == PART:
                        q.put((p * PART + reported[p], p * PART + landed[p]))
                        reported[p] = landed[p]

    t0 = time.perf_counter()
    with ThreadPoolExecutor(8) as ex:
        list(ex.map(work, range(8)))
    t_write = time.perf_counter() - t0
    q.put(None)
    th.join()
    s.synchronize()
    return round(t_write * 1e3, 1), round((time.perf_counter() - t0) * 1e3, 1)


run(False)
run(True)
print(json.dumps({"step": STEP, "writers_alone_ms": run(False), "writers_with_stager_ms_and_total": run(True),
                  "writers_alone_again_ms": run(False)}))
