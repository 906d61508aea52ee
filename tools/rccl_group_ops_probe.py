"""RCCL grouped point-to-point probe: does one ncclGroupStart/End with thousands of ncclSend/ncclRecv
pairs (the zero-copy TeraSort round: reducers x maps slices per peer, `csrc/gpu/exchange.cc`) complete,
deliver the bytes, and how does its time compare with one message per peer (the packed mode)?

A single GPU cannot host two RCCL ranks (RCCL rejects a duplicate device), so this runs one rank that
sends to and receives from itself: the same group/op bookkeeping and kernel-plan splitting as a
multi-rank round, with the bytes moved by RCCL's local path instead of xGMI. It checks op-count
scalability and correctness of the grouped API, not link bandwidth.

    python tools/rccl_group_ops_probe.py --total-mb 7168 --ops 7,512,3584
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import time

import torch


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


def load_rccl():
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    lib = ctypes.CDLL(path if os.path.exists(path) else "librccl.so")
    lib.ncclGetErrorString.restype = ctypes.c_char_p
    return lib


def check(lib, r, what):
    if r != 0:
        raise RuntimeError(f"{what}: RCCL error {r} {lib.ncclGetErrorString(r).decode()}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total-mb", type=int, default=7168)
    ap.add_argument("--ops", default="7,512,3584")
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    lib = load_rccl()
    uid = UniqueId()
    check(lib, lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
    comm = ctypes.c_void_p()
    check(lib, lib.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0), "ncclCommInitRank")
    total = a.total_mb << 20
    src = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    stream = torch.cuda.Stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    for n_ops in [int(x) for x in a.ops.split(",")]:
        per = (total // n_ops) & ~255
        dst.zero_()
        times = []
        for it in range(a.iters + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            check(lib, lib.ncclGroupStart(), "ncclGroupStart")
            for k in range(n_ops):
                s = ctypes.c_void_p(src.data_ptr() + k * per)
                d = ctypes.c_void_p(dst.data_ptr() + k * per)
                check(lib, lib.ncclSend(s, ctypes.c_size_t(per), 1, 0, comm, sp), "ncclSend")
                check(lib, lib.ncclRecv(d, ctypes.c_size_t(per), 1, 0, comm, sp), "ncclRecv")
            t_issue = time.perf_counter() - t0
            check(lib, lib.ncclGroupEnd(), "ncclGroupEnd")
            stream.synchronize()
            dt = time.perf_counter() - t0
            if it > 0:
                times.append((dt, t_issue))
        ok = bool(torch.equal(src[: per * n_ops], dst[: per * n_ops]))
        best = min(times)
        print(json.dumps({"ops_per_group": n_ops, "bytes_per_op": per, "bytes": per * n_ops, "ok": ok,
                          "ms": round(best[0] * 1e3, 2), "issue_ms": round(best[1] * 1e3, 2),
                          "GBps": round(per * n_ops / best[0] / 1e9, 1)}), flush=True)
        if not ok:
            raise SystemExit("data mismatch")
    lib.ncclCommDestroy(comm)


if __name__ == "__main__":
    main()
