"""How long does another process take to map a device allocation of a given size over hipIpc (dmabuf
IPC on this image), and can it read the last byte? The multi-rank UdaBridge API path maps every other
rank's map-output store this way (csrc/gpu/device_ptr.cc).

    python tools/ipc_size_probe.py 1 2 3 4 6      # sizes in GiB
"""
from __future__ import annotations

import ctypes
import json
import subprocess
import sys
import time

CHILD = r"""
import ctypes, sys, time, json
hip = ctypes.CDLL("libamdhip64.so")
class H(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]
h = H()
ctypes.memmove(ctypes.byref(h), bytes.fromhex(sys.argv[1]), 64)
size = int(sys.argv[2])
hip.hipSetDevice(0)
t0 = time.perf_counter()
p = ctypes.c_void_p()
rc = hip.hipIpcOpenMemHandle(ctypes.byref(p), h, 1)
t1 = time.perf_counter()
out = ctypes.c_uint64(0)
rc2 = hip.hipMemcpy(ctypes.byref(out), ctypes.c_void_p(p.value + size - 8), ctypes.c_size_t(8), 2) if rc == 0 else -1
t2 = time.perf_counter()
print(json.dumps({"open_rc": rc, "open_ms": round((t1 - t0) * 1e3, 1), "read_rc": rc2,
                  "read_ms": round((t2 - t1) * 1e3, 1), "last_word": hex(out.value)}), flush=True)
if rc == 0:
    hip.hipIpcCloseMemHandle(p)
"""


def main():
    import torch
    hip = ctypes.CDLL("libamdhip64.so")

    class H(ctypes.Structure):
        _fields_ = [("reserved", ctypes.c_char * 64)]

    for gib in [float(x) for x in sys.argv[1:]] or [1, 2, 3, 4]:
        size = int(gib * (1 << 30)) // 8 * 8
        t = torch.empty(size // 8, dtype=torch.int64, device="cuda")
        t[-1] = 0x1234567890
        torch.cuda.synchronize()
        # torch's caching allocator may hand out part of a bigger block: export the block base
        base, rng = ctypes.c_void_p(), ctypes.c_size_t()
        hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(rng), ctypes.c_void_p(t.data_ptr()))
        h = H()
        t0 = time.perf_counter()
        rc = hip.hipIpcGetMemHandle(ctypes.byref(h), base)
        get_ms = (time.perf_counter() - t0) * 1e3
        off = t.data_ptr() - base.value
        try:
            r = subprocess.run([sys.executable, "-c", CHILD, bytes(h).hex(), str(off + size)], capture_output=True,
                               text=True, timeout=60)
            child = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-300:]
        except subprocess.TimeoutExpired:
            child = "TIMEOUT (60 s)"
        print(json.dumps({"gib": gib, "block_bytes": rng.value, "get_rc": rc, "get_ms": round(get_ms, 1),
                          "child": child}), flush=True)
        del t
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
