#!/usr/bin/env python3
"""Which processes can map a device allocation over hipIpc (dmabuf IPC on this image)? The exporter
(this process, torch allocation) hands its handle to: a child started with subprocess (fork+exec), a
child started with os.posix_spawn with default signal dispositions (the node daemon's spawn), and a
grandchild. One JSON line per importer: open_rc (0 = mapped), read_rc, the last word read.

    python tools/ipc_lineage_probe.py
"""
from __future__ import annotations

import ctypes
import json
import os
import signal
import subprocess
import sys

IMPORTER = r"""
import ctypes, sys, json, os, subprocess
hip = ctypes.CDLL("libamdhip64.so")
class H(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]
h = H()
ctypes.memmove(ctypes.byref(h), bytes.fromhex(sys.argv[1]), 64)
size, who = int(sys.argv[2]), sys.argv[3]
hip.hipSetDevice(0)
p = ctypes.c_void_p()
rc = hip.hipIpcOpenMemHandle(ctypes.byref(p), h, 1)
out = ctypes.c_uint64(0)
rc2 = hip.hipMemcpy(ctypes.byref(out), ctypes.c_void_p(p.value + size - 8), ctypes.c_size_t(8), 2) if rc == 0 else -1
print(json.dumps({"importer": who, "pid": os.getpid(), "ppid": os.getppid(), "open_rc": rc, "read_rc": rc2,
                  "last_word": hex(out.value)}), flush=True)
if rc == 0:
    hip.hipIpcCloseMemHandle(p)
if who == "child-then-grandchild":
    subprocess.run([sys.executable, "-c", sys.argv[4], sys.argv[1], sys.argv[2], "grandchild"], check=False)
"""


def main() -> int:
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    size = 64 << 20
    t = torch.full((size // 8,), 0x1122334455667788, dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()

    class H(ctypes.Structure):
        _fields_ = [("reserved", ctypes.c_char * 64)]
    h = H()
    base = ctypes.c_void_p()
    sz = ctypes.c_size_t()
    hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(sz), ctypes.c_void_p(t.data_ptr()))
    rc = hip.hipIpcGetMemHandle(ctypes.byref(h), base)
    print(json.dumps({"exporter": os.getpid(), "get_rc": rc, "alloc_bytes": sz.value,
                      "env_ipc_legacy": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")}), flush=True)
    hexh = bytes(h.reserved).hex()
    n = str(sz.value)
    subprocess.run([sys.executable, "-c", IMPORTER, hexh, n, "child(subprocess)"], check=False, timeout=120)
    attr = {"setsigdef": tuple(s for s in signal.valid_signals() if s not in (signal.SIGKILL, signal.SIGSTOP)),
            "setsigmask": ()}
    pid = os.posix_spawn(sys.executable, [sys.executable, "-c", IMPORTER, hexh, n, "child(posix_spawn, sigdef)"],
                         dict(os.environ), **attr)
    os.waitpid(pid, 0)
    subprocess.run([sys.executable, "-c", IMPORTER, hexh, n, "child-then-grandchild", IMPORTER], check=False,
                   timeout=240)
    del t
    return 0


if __name__ == "__main__":
    sys.exit(main())
