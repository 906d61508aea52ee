#!/usr/bin/env python3
"""J2C consumer threading A/B: one reduce task consuming 1 GiB of 1 MiB TeraSort buffers (out of
cache) and one 1 MiB buffer 2000 times (cached), walks inline vs on the reduce task's own thread."""
import time, numpy as np, sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from uda_amd import native
from uda_amd.utils.ifile import encode_stream, text
n = native()
# 1 MiB of 104-byte TeraSort records (whole records), replicated into a 1 GiB source (out of cache)
rec = encode_stream([(text(b"%010d" % i), text(b"V" * 90)) for i in range(10082)])[:-2]
one = np.frombuffer(rec, dtype=np.uint8)
src = np.tile(one, 1024)  # ~1 GiB
blen = len(one)
for threaded in (False, True, False, True):
    s = n.J2CSink(1, 1 << 20, threaded)
    mv = memoryview(src)
    t0 = time.perf_counter()
    for i in range(1024):
        s.consume(0, mv[i * blen:(i + 1) * blen])
    s.flush()
    dt = time.perf_counter() - t0
    print("threaded" if threaded else "inline  ", round(src.nbytes / dt / 1e9, 2), "GB/s", s.records(0))
# cache-resident: same 1 MiB buffer 2000 times
for threaded in (False, True):
    s = n.J2CSink(1, 1 << 20, threaded)
    t0 = time.perf_counter()
    s.consume(0, one, 2000)
    s.flush()
    dt = time.perf_counter() - t0
    print("cached", "threaded" if threaded else "inline  ", round(blen * 2000 / dt / 1e9, 2), "GB/s")
t0 = time.perf_counter(); x = src.copy(); dt = time.perf_counter() - t0
print("numpy copy 1GiB", round(src.nbytes / dt / 1e9, 2), "GB/s")
