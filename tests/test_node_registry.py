"""CPU tier: the node-local registry behind mapred.uda.gpu.device=auto and the HBM byte budget
(uda/node_registry.h, csrc/gpu/hbm_ledger.h), with real processes.

Placement: a reduce task takes the visible GPU with the fewest live tasks on the node (fake device
keys: 1, 2 and 8 GPUs); 16 concurrent registrant processes spread evenly; a registrant that dies
without releasing is reclaimed by the next caller. Budget: reservations wait for bytes another
process frees, idle pooled objects are trimmed largest-first under pressure, and a working set
larger than the headroom (budget minus resident stores) is refused at once.

Reference analogue: one NetMerger per reduce-task process (src/Merger/reducer.h:137), every IB
device of the node mapped (src/DataNet/RDMAComm.cc:156-176), buffers sized from the shuffle memory
budget (src/Merger/reducer.cc:102-120, 453-496)."""
import multiprocessing as mp
import os
import secrets
import time

import pytest

GB = 1 << 30


def _name():
    return f"udareg.{os.getpid()}.{secrets.token_hex(4)}"


@pytest.fixture()
def reg():
    import uda_amd
    n = uda_amd.native()
    r = n.NodeRegistry(_name())
    yield n, r
    r.unlink()


@pytest.mark.parametrize("ndev", [1, 2, 8])
def test_placement_spreads_over_devices(reg, ndev):
    n, r = reg
    keys = [f"0000:{i:02x}:00.0" for i in range(ndev)]
    slots = []
    counts = [0] * ndev
    for t in range(2 * ndev + 1):
        idx, slot = r.place_task(keys, f"attempt_r_{t}")
        counts[idx] += 1
        slots.append(slot)
    assert max(counts) - min(counts) <= 1, counts
    assert sum(r.usage(k)["tasks"] for k in keys) == 2 * ndev + 1
    # a released slot's device is the next one chosen
    r.release(slots[0])
    idx, _ = r.place_task(keys, "again")
    assert idx == 0
    # ties broken by bytes held on the node: the emptier GPU wins
    if ndev > 1:
        r2 = n.NodeRegistry(r.name)
        for k in keys:
            r2.usage(k)
        keys2 = keys[:2]
        t0 = r.usage(keys2[0])["tasks"]
        t1 = r.usage(keys2[1])["tasks"]
        if t0 == t1:
            r.set_bytes(keys2[0], 10 * GB)
            idx, _ = r.place_task(keys2, "bytes-tie")
            assert idx == 1


def test_pinned_tasks_count_for_auto(reg):
    _, r = reg
    keys = ["gpuA", "gpuB"]
    r.add_task("gpuA", "pinned-1")
    r.add_task("gpuA", "pinned-2")
    idx, _ = r.place_task(keys, "auto")
    assert idx == 1


def _register_and_hold(name, keys, q, go, hold):
    import uda_amd
    n = uda_amd.native()
    r = n.NodeRegistry(name)
    go.wait(30)  # every registrant places at the same moment
    idx, slot = r.place_task(keys, f"proc-{os.getpid()}")
    q.put(idx)
    hold.wait(60)
    r.release(slot)


def test_concurrent_registrants_balance(reg):
    _, r = reg
    ctx = mp.get_context("spawn")
    keys = [f"dev{i}" for i in range(8)]
    q, go, hold = ctx.Queue(), ctx.Event(), ctx.Event()
    ps = [ctx.Process(target=_register_and_hold, args=(r.name, keys, q, go, hold)) for _ in range(16)]
    for p in ps:
        p.start()
    time.sleep(1.0)
    go.set()
    got = [q.get(timeout=60) for _ in ps]
    counts = [got.count(i) for i in range(8)]
    assert counts == [2] * 8, counts
    assert sum(r.usage(k)["tasks"] for k in keys) == 16
    hold.set()
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    assert sum(r.usage(k)["tasks"] for k in keys) == 0


def _die_registered(name, keys, q):
    import uda_amd
    n = uda_amd.native()
    r = n.NodeRegistry(name)
    idx, _ = r.place_task(keys, "doomed")
    r.set_bytes(keys[idx], 7 * GB, 5 * GB)
    q.put(idx)
    q.close()
    q.join_thread()  # the index reached the parent
    os._exit(3)  # no release, no destructor: like a killed reduce task JVM


def test_dead_registrant_reclaimed(reg):
    _, r = reg
    ctx = mp.get_context("spawn")
    keys = ["gpu0", "gpu1"]
    q = ctx.Queue()
    p = ctx.Process(target=_die_registered, args=(r.name, keys, q))
    p.start()
    idx = q.get(timeout=60)
    p.join(30)
    assert p.exitcode == 3
    # its slot still shows until a caller looks for dead processes; place_task reaps first
    new_idx, _ = r.place_task(keys, "survivor")
    assert new_idx == 0  # the dead task no longer counts on gpu{idx}; ties -> lowest index
    assert r.reclaimed >= 2  # the task and its bytes entry
    assert r.usage(keys[idx])["bytes"] == 0 and r.usage(keys[idx])["resident"] == 0


def test_process_liveness_helpers():
    import uda_amd
    n = uda_amd.native()
    me = os.getpid()
    st = n.process_start_ticks(me)
    assert st > 0
    assert n.process_running(me, st)
    assert not n.process_running(me, st + 1)  # same pid, other process (pid reuse)
    assert not n.process_running(2 ** 22 + 12345, 0)


# ------------------------------------------------------------------------------ HBM byte budget
# Fake devices (no HIP): ids >= 100, keys unique per test; the ledger publishes into the registry
# named by UDA_NODE_REGISTRY, so every test runs in fresh processes that share that name.

def _ledger_proc(fn, name, args, q):
    os.environ["UDA_NODE_REGISTRY"] = name
    try:
        import uda_amd
        q.put(fn(uda_amd.native(), *args))
    except BaseException as e:  # noqa: BLE001
        q.put(f"EXC:{type(e).__name__}:{e}")


def _in_proc(fn, *args, name=None, timeout=120):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_ledger_proc, args=(fn, name or _name(), args, q))
    p.start()
    v = q.get(timeout=timeout)
    p.join(30)
    return v


def _budget_and_trim(n, key):
    d = 100
    n.hbm_fake_device(d, 100 * GB, key)
    n.hbm_configure(d, 50 * GB)  # bytes (> 1)
    n.hbm_alloc(d, 10 * GB, resident=True)  # a MOF store: stays
    n.hbm_fake_pool(d, [8 * GB, 2 * GB, 12 * GB])  # idle pooled workspaces (22 GB)
    out = {"headroom": n.hbm_headroom(d)}
    r = n.hbm_reserve(d, 25 * GB, 5.0)  # needs 7 GB of the pool trimmed: the 12 GB object goes
    s = n.hbm_stats(d)
    out.update(granted=r.granted, trimmed=s["trimmed"], used=s["used"], reserved=s["reserved"])
    r.alloc(20 * GB)  # drawn from the reservation: no overrun
    s = n.hbm_stats(d)
    out.update(over_after_draw=s["over"], reserved_after_draw=s["reserved"])
    r.release()
    out["reserved_after_release"] = n.hbm_stats(d)["reserved"]
    try:
        n.hbm_reserve(d, 45 * GB, 1.0)  # > headroom (50 - 10 resident): refused at once
        out["too_big"] = "granted"
    except Exception as e:  # noqa: BLE001
        out["too_big"] = str(e)
    n.hbm_alloc(d, 45 * GB)  # outside any reservation, past the budget: allowed, but counted
    out["over_outside"] = n.hbm_stats(d)["over"]
    n.hbm_free(d, 45 * GB)
    n.hbm_configure(d, 0.5)  # a fraction of the device
    out["budget_fraction"] = n.hbm_stats(d)["budget"]
    return out


def test_hbm_budget_trims_idle_pools_and_refuses_oversize():
    o = _in_proc(_budget_and_trim, "fake-budget-" + secrets.token_hex(3))
    assert not isinstance(o, str), o
    assert o["headroom"] == 40 * GB
    assert o["granted"] == 25 * GB
    assert o["trimmed"] == 12 * GB  # largest idle object first, and only as much as needed
    assert o["used"] == 10 * GB + 10 * GB and o["reserved"] == 25 * GB
    assert o["over_after_draw"] == 0 and o["reserved_after_draw"] == 5 * GB
    assert o["reserved_after_release"] == 0
    assert "exceeds the HBM budget headroom" in o["too_big"], o["too_big"]
    assert o["budget_fraction"] == 50 * GB
    assert o["over_outside"] == 45 * GB  # reported as hbm_over_budget_bytes in the bench JSON


def _hold_bytes(n, key, go_file, hold_s):
    d = 101
    n.hbm_fake_device(d, 100 * GB, key)
    n.hbm_alloc(d, 60 * GB)  # another process's working set
    open(go_file, "w").close()
    time.sleep(hold_s)
    n.hbm_free(d, 60 * GB)
    time.sleep(0.5)
    return "freed"


def _wait_for_bytes(n, key, go_file):
    d = 101
    n.hbm_fake_device(d, 100 * GB, key)
    n.hbm_configure(d, 80 * GB)
    t0 = time.time()
    while not os.path.exists(go_file) and time.time() - t0 < 60:
        time.sleep(0.01)
    before = n.hbm_stats(d)["node_bytes"]
    r = n.hbm_reserve(d, 40 * GB, 30.0)  # 60 + 40 > 80: waits for the other process
    return {"node_before": before, "wait_ms": r.wait_ms, "granted": r.granted}


def test_hbm_reservation_waits_for_another_process(tmp_path):
    ctx = mp.get_context("spawn")
    name = _name()
    key = "fake-node-" + secrets.token_hex(3)
    go = str(tmp_path / "go")
    q1, q2 = ctx.Queue(), ctx.Queue()
    p1 = ctx.Process(target=_ledger_proc, args=(_hold_bytes, name, (key, go, 1.5), q1))
    p2 = ctx.Process(target=_ledger_proc, args=(_wait_for_bytes, name, (key, go), q2))
    p1.start()
    p2.start()
    o = q2.get(timeout=90)
    assert q1.get(timeout=90) == "freed"
    p1.join(30)
    p2.join(30)
    assert not isinstance(o, str), o
    assert o["node_before"] == 60 * GB  # the other process's bytes, seen through the registry
    assert o["granted"] == 40 * GB
    assert o["wait_ms"] > 800  # granted only once the holder freed its 60 GB


def _untracked_headroom(n, key):
    d = 102
    n.hbm_fake_device(d, 100 * GB, key)
    n.hbm_configure(d, 50 * GB)
    n.hbm_alloc(d, 10 * GB, resident=True)  # the provider's MOF store
    n.hbm_fake_untracked(d, 15 * GB)  # HIP runtime, code objects, allocations outside libuda
    out = {"headroom": n.hbm_headroom(d)}
    t0 = time.time()
    try:
        n.hbm_reserve(d, 30 * GB, 30.0)  # fits the ledger (10 + 30 <= 50), never the device (15 + 10 + 30 > 50)
        out["big"] = "granted"
    except Exception as e:  # noqa: BLE001
        out["big"] = str(e)
    out["big_s"] = time.time() - t0
    r = n.hbm_reserve(d, 25 * GB, 5.0)  # exactly the headroom: granted at once
    out["granted"] = r.granted
    return out


def test_hbm_headroom_counts_untracked_device_memory():
    """headroom() is what round sizing shrinks to; it must include the device memory no ledger
    tracks, or a task sized from it passes the headroom check and then polls until the 1800 s timeout
    (blocking every later reservation of the device behind it, FIFO)."""
    o = _in_proc(_untracked_headroom, "fake-untracked-" + secrets.token_hex(3))
    assert not isinstance(o, str), o
    assert o["headroom"] == 25 * GB
    assert "exceeds the HBM budget headroom" in o["big"] and o["big_s"] < 5, o
    assert o["granted"] == 25 * GB
