"""CPU tier: the node-local shared-memory control plane of the IPC exchange (uda/shm_group.h) with
real rank processes — barrier, chunked all-to-all of counts, round counters, allocation tables,
abort propagation and dead-peer detection (a crashed rank must make its peers throw, not hang).

Reference analogue: RDMA-CM connection setup + SEND/RECV control messages and credits
(src/DataNet/RDMAClient.cc:215-356, src/DataNet/RDMAComm.cc:707-752)."""
import multiprocessing as mp
import os
import secrets
import time

import pytest

OUT, IN, DONE, USER = 0, 1, 2, 3


def _name():
    return f"udatest.{os.getpid()}.{secrets.token_hex(4)}"


def _worker(fn, name, rank, world, q):
    try:
        import uda_amd
        n = uda_amd.native()
        q.put((rank, fn(n, name, rank, world)))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, f"EXC:{type(e).__name__}:{e}"))


def _run(fn, world, timeout=120):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = _name()
    ps = [ctx.Process(target=_worker, args=(fn, name, r, world, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    t0 = time.time()
    while len(out) < world and time.time() - t0 < timeout:
        try:
            r, v = q.get(timeout=1)
            out[r] = v
        except Exception:  # noqa: BLE001
            if all(not p.is_alive() for p in ps) and q.empty():
                break
    for p in ps:
        p.join(timeout=10)
        if p.is_alive():
            p.kill()
    assert not os.path.exists(f"/dev/shm/{name}"), "segment left behind in /dev/shm"
    return [out.get(r) for r in range(world)]


def _collectives(n, name, rank, world):
    g = n.ShmGroup(name, rank, world, mailbox_bytes=4096, outbox_bytes=4096, timeout_s=60)
    for _ in range(5):
        g.barrier()
    # 1000 int64 per peer through a 4 KiB mailbox: many chunks
    per = 1000
    send = [rank * 1_000_000 + p * 10_000 + i for p in range(world) for i in range(per)]
    recv = g.alltoall(send)
    ok = all(recv[p * per + i] == p * 1_000_000 + rank * 10_000 + i for p in range(world) for i in range(per))
    # counters: round-robin publish / wait
    for k in range(1, 20):
        g.publish(OUT, k)
        g.wait_at_least(OUT, -1, k)
    blob = bytes([rank]) * 64
    aid = g.publish_alloc(blob, 1000 + rank)
    g.barrier()
    peers = [g.read_alloc(p, aid) for p in range(world)]
    ok_alloc = all(b == bytes([p]) * 64 and sz == 1000 + p for p, (b, sz) in enumerate(peers))
    missing = g.read_alloc((rank + 1) % world, 5) is None
    g.barrier()
    return ok and ok_alloc and missing


def _abort(n, name, rank, world):
    g = n.ShmGroup(name, rank, world, timeout_s=60)
    if rank == 1:
        time.sleep(0.3)
        g.abort("injected failure")
        return "aborted"
    try:
        g.wait_at_least(USER, 1, 1)  # rank 1 never publishes
        return "no-throw"
    except Exception as e:  # noqa: BLE001
        return str(e)


def _dead_peer(n, name, rank, world):
    g = n.ShmGroup(name, rank, world, timeout_s=60)
    if rank == 2:
        os._exit(3)  # crash without any cleanup
    t0 = time.time()
    try:
        g.barrier()
        return "no-throw"
    except Exception as e:  # noqa: BLE001
        return f"{time.time() - t0:.1f}s {e}"


def _timeout(n, name, rank, world):
    g = n.ShmGroup(name, rank, world, timeout_s=1.0)
    if rank == 0:
        try:
            g.wait_at_least(USER, 1, 7)
            return "no-throw"
        except Exception as e:  # noqa: BLE001
            return str(e)
    time.sleep(2.5)  # alive but silent past the timeout
    return "slept"


def test_collectives_three_ranks():
    assert _run(_collectives, 3) == [True, True, True]


def test_abort_wakes_waiters():
    res = _run(_abort, 3)
    assert res[1] == "aborted"
    for r in (0, 2):
        assert "aborted" in res[r] and "injected failure" in res[r], res


def test_dead_peer_detected():
    res = _run(_dead_peer, 3)
    assert res[2] is None  # crashed
    for r in (0, 1):
        assert "died" in res[r], res
        assert float(res[r].split("s ")[0]) < 10


def test_timeout_aborts():
    res = _run(_timeout, 2)
    assert "timed out" in res[0], res


def test_bad_arguments(native):
    with pytest.raises(Exception):
        native.ShmGroup(_name(), 2, 2)
    with pytest.raises(Exception):
        native.ShmGroup("bad/name", 0, 1)
    g = native.ShmGroup(_name(), 0, 1)  # world 1: attach is immediate
    g.barrier()
    assert g.alltoall([1, 2, 3]) == [1, 2, 3]
