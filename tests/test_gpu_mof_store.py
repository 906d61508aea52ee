"""GPU: lifetime of the provider's HBM store of MOF files (csrc/gpu/mof_cache.h).

A descriptor handed to a reducer is a reference the reducer holds until it releases it: an entry
with a live holder is never evicted, however long ago it was served and however full the budget;
a released, finished-job, or dead holder's entry is evictable. Reducers release their descriptors
when their merge is done (a release message on the fetch transport), so a job's store drains.

Reference: chunks are freed only when the SEND that used them completed, and the fd cache is
refcounted by in-flight reads (src/DataNet/RDMAServer.cc:200-213, src/MOFServer/IndexInfo.cc:195-233,
276-301)."""
import json
import os
import time

import pytest

from uda_amd.bridge import UdaProvider, run_reduce
from uda_amd.utils import datagen
from uda_amd.utils.mof import encode_partitions

pytestmark = pytest.mark.gpu
GPU = {"mapred.uda.merge.backend": "gpu"}
MB = 1 << 20


def _files(tmp_path, n, size):
    paths = []
    for i in range(n):
        p = tmp_path / f"mof{i}.out"
        p.write_bytes(os.urandom(size))
        paths.append(str(p))
    return paths


def test_held_entry_outlives_its_lease_under_budget_pressure(require_gpu, native, tmp_path):
    size = 24 * MB + 4096 * 3  # not a multiple of the chunk: a short last read
    f = _files(tmp_path, 3, size)
    store = native.MofStore(capacity=2 * size + MB, devices=[0], lease_s=0.5, chunk_bytes=4 * MB)
    me = native.reducer_holder_id("attempt_r_000000_0")  # this process: alive
    ok, why, a0, n0, _ = store.acquire("job", f[0], me)
    assert ok and n0 == size, why
    assert native.device_read(a0, size) == open(f[0], "rb").read()  # every chunk landed in order
    ok, _, _, _, _ = store.acquire("job", f[1], me)
    assert ok
    time.sleep(1.2)  # past the lease: a held entry stays anyway
    ok, why, _, _, _ = store.acquire("job", f[2], "other-reducer")
    assert not ok and "held" in why, why
    st = store.stats()
    assert st["evictions"] == 0 and st["holders"] == 2 and st["declined"] == 1, st
    assert native.device_read(a0, 4096) == open(f[0], "rb").read(4096)  # still resident and intact
    store.release(f[0], me)
    ok, why, a2, _, _ = store.acquire("job", f[2], "other-reducer")
    assert ok, why
    assert native.device_read(a2, size) == open(f[2], "rb").read()
    st = store.stats()
    assert st["evictions"] == 1 and st["releases"] == 1 and st["loads"] == 3, st


def test_a_job_does_not_evict_its_own_recently_served_files(require_gpu, native, tmp_path):
    """mapred.uda.provider.hbm.idle.evict.s: a job whose MOFs outgrow the store reads them in waves; a file
    it was served recently is not evicted to load another of its files (the next wave would reload it),
    while another job, or the same job once the file has been idle that long, may take the space."""
    size = 8 * MB
    f = _files(tmp_path, 4, size)
    store = native.MofStore(capacity=2 * size + MB, devices=[0], idle_evict_s=0.6)
    for p in f[:2]:
        assert store.acquire("j", p, "a")[0]
        store.release(p, "a")
    ok, why, _, _, _ = store.acquire("j", f[2], "b")
    assert not ok and "recently served" in why, why
    ok, why, _, _, _ = store.acquire("k", f[3], "c")  # another job: the LRU file of j goes
    assert ok, why
    assert store.stats()["evictions"] == 1
    time.sleep(0.8)
    ok, why, a2, _, _ = store.acquire("j", f[2], "b")  # j's remaining file has been idle long enough
    assert ok, why
    assert native.device_read(a2, size) == open(f[2], "rb").read()
    st = store.stats()
    assert st["evictions"] == 2 and st["declined"] == 1, st


@pytest.mark.parametrize("cached_read", [True, False])
def test_files_in_the_page_cache_are_read_through_it(require_gpu, native, tmp_path, cached_read):
    """mapred.uda.provider.hbm.cached.read: a MOF file whose pages are all in the page cache (just written)
    is loaded with buffered reads instead of O_DIRECT (which would read it from the disk again); either way
    every byte lands."""
    size = 24 * MB + 4096 * 3 + 100  # a short, unaligned last read
    f = _files(tmp_path, 2, size)
    for p in f:
        open(p, "rb").read()  # (surely) in the page cache
    store = native.MofStore(capacity=4 * size, devices=[0], chunk_bytes=4 * MB, cached_read=cached_read)
    for p in f:
        ok, why, a, n, _ = store.acquire("job", p, "r")
        assert ok and n == size, why
        assert native.device_read(a, size) == open(p, "rb").read()
    assert store.stats()["cached_reads"] == (2 if cached_read else 0)


def test_dead_or_foreign_holders_are_dropped(require_gpu, native, tmp_path):
    size = 8 * MB
    f = _files(tmp_path, 3, size)
    store = native.MofStore(capacity=2 * size + MB, devices=[0], lease_s=0.5)
    dead = f"{native.node_id()}:999999:1:attempt_r_1"  # this node, a process that is gone
    foreign = "0123456789abcdef:4242:7:attempt_r_2"  # another node: only its lease protects it
    assert store.acquire("job", f[0], dead)[0]
    assert store.acquire("job", f[1], foreign)[0]
    # the foreign holder fetched just now: its entry stays; the dead holder's entry goes
    ok, why, _, _, _ = store.acquire("job", f[2], "x")
    assert ok, why
    st = store.stats()
    assert st["evictions"] == 1 and st["holders_reaped"] == 1, st
    time.sleep(1.0)  # the foreign holder's lease runs out
    store.release(f[2], "x")
    ok, why, _, _, _ = store.acquire("job", f[0], "y")
    assert ok, why
    assert store.stats()["holders_reaped"] == 2


def test_reduce_tasks_release_their_descriptors(require_gpu, tmp_path):
    """A job's reduce tasks fetch descriptors of Hadoop-written MOFs and release them when merged:
    afterwards nothing is held, and another job can take the HBM without waiting for JOB_OVER."""
    from uda_amd.utils.mof import write_mof
    maps = datagen.terasort(num_maps=4, reducers=2, rows_per_map=3000, seed=31)
    size = sum(len(b) for b in datagen.streams(maps)[0]) + 4096
    p = UdaProvider(conf={"mapred.uda.provider.hbm.bytes": 5 * size})
    try:
        ids = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_job_9_0200_m_{i:06d}_0"
            path, _ = write_mof(str(tmp_path), mid, parts)
            p.add_mof_file("job_9_0200", mid, path)
            ids.append(mid)
        conf = dict(GPU, **{"mapred.uda.gpu.fetch": "device"})
        for r in range(2):
            recs, st, _ = run_reduce("h", "job_9_0200", ids, r, datagen.TEXT, conf=conf)
            assert len(recs) == sum(len(m[r]) for m in maps)
            assert st["device_descriptors"] == 4, st
        hs = json.loads(p.stats())["hbm_store"]
        assert hs["holders"] == 0 and hs["releases"] >= 8 and hs["loads"] == 4, hs
        # a second job's MOFs fit only by evicting the first job's (released, job still running)
        ids2 = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_job_9_0201_m_{i:06d}_0"
            path, _ = write_mof(str(tmp_path / "j2"), mid, parts)
            p.add_mof_file("job_9_0201", mid, path)
            ids2.append(mid)
        recs, st, _ = run_reduce("h", "job_9_0201", ids2, 0, datagen.TEXT, conf=conf)
        assert st["device_descriptors"] == 4 and st["host_fetched_bytes"] == 0, st
        hs = json.loads(p.stats())["hbm_store"]
        assert hs["evictions"] >= 3 and hs["declined"] == 0, hs
    finally:
        p.close()


def test_empty_partitions_on_the_generic_device_path(require_gpu):
    """Every partition holds only its EOF marker (BytesWritable keys: the generic merge, not FIXED10):
    the task must end with an EOF-only delivery instead of waiting for a round that never merges."""
    p = UdaProvider()
    try:
        ids = []
        for i, parts in enumerate(datagen.streams([[[], []] for _ in range(5)])):  # EOF markers only
            mid = f"attempt_job_9_0202_m_{i:06d}_0"
            data, index = encode_partitions(parts, None)
            p.add_mof_device("job_9_0202", mid, data, index, device=0)
            ids.append(mid)
        conf = dict(GPU, **{"mapred.uda.gpu.fetch": "device", "mapred.uda.gpu.round.bytes": 1 << 20})
        t0 = time.time()
        recs, st, _ = run_reduce("h", "job_9_0202", ids, 1, datagen.BYTES, conf=conf)
        assert recs == [] and st["records"] == 0 and st["merge_path"] == "device-generic", st
        assert time.time() - t0 < 60
    finally:
        p.close()


@pytest.mark.parametrize("service", [False, True])
def test_bench_node_shape_small(require_gpu, service):
    """bench.py --api --node: the provider in its own process, every reduce task a fresh uda_reduce_task
    process mapping the provider's HBM over hipIpc (validated wave, descriptors only); with
    --node-service the NetMergers run in the provider process and the task processes read the merged
    buffers in place from its shared pinned rings (zero-copy)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--api", "--node", "--reducers", "3", "--rows-per-gpu",
           "3000000", "--maps-per-gpu", "6", "--steps", "1", "--warmup", "1", "--node-service" if service else "--no-node-service"]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["validated"] is True, out
    t0 = out["task0_stats"]
    assert t0["device_descriptors"] == 6 and t0["host_fetched_bytes"] == 0 and t0["gpu_device"] == 0, t0
    assert out["node"]["task_ms_median"]["fetch_to_eof_ms"] > 0
    if service:
        ms = out["provider"]["merge_service"]
        assert t0.get("merge_service") is True and ms["sessions"] >= 6, ms
        assert ms["zero_copy_buffers"] > ms["bounced_buffers"], ms


def test_hbm_budget_counts_untracked_device_memory(require_gpu, native):
    """A reservation is checked against what the device reports in use, not only the ledger's own
    allocations: HBM taken outside the ledger (here a torch tensor) leaves less room under the budget."""
    import torch
    d = 0
    native.hbm_stats(d)  # initializes the device's ledger entry
    free, total = torch.cuda.mem_get_info(d)
    used = total - free
    try:
        native.hbm_configure(d, float(used + (6 << 30)))  # budget: what is in use now + 6 GiB
        r = native.hbm_reserve(d, 2 << 30, 10.0)  # fits
        del r
        blob = torch.empty(5 << 30, dtype=torch.uint8, device=f"cuda:{d}")  # untracked 5 GiB
        with pytest.raises(Exception, match="HBM"):
            native.hbm_reserve(d, 2 << 30, 1.0)  # 5 + 2 > 6 GiB: waits, then gives up
        del blob
        torch.cuda.empty_cache()
        r = native.hbm_reserve(d, 2 << 30, 10.0)  # room again once the untracked memory is gone
        del r
        assert native.hbm_stats(d)["device_peak"] >= used + (5 << 30)
    finally:
        native.hbm_configure(d, 0.0)  # back to the default fraction


def test_store_declines_after_an_injected_loader_setup_failure(require_gpu, native, tmp_path, monkeypatch):
    """a loader whose setup fails (UDA_FAULT_STORE_SETUP) answers its queued request with a
    decline and declines every later one at once, instead of reading an empty slot table."""
    f = _files(tmp_path, 1, 4 * MB)
    monkeypatch.setenv("UDA_FAULT_STORE_SETUP", "1")
    store = native.MofStore(capacity=64 * MB, devices=[0])
    t0 = time.time()
    ok, why, _, _, _ = store.acquire("job", f[0], "r1")
    assert not ok and "injected" in why, why
    time.sleep(0.3)
    ok, why, _, _, _ = store.acquire("job", f[0], "r2")
    assert not ok and "unavailable" in why, why
    assert time.time() - t0 < 30
    monkeypatch.delenv("UDA_FAULT_STORE_SETUP")
    store2 = native.MofStore(capacity=64 * MB, devices=[0])  # a new store's loader starts normally
    ok, why, a, n, _ = store2.acquire("job", f[0], "r3")
    assert ok and n == 4 * MB, why


def test_bench_node_files_default_configuration(require_gpu, tmp_path):
    """bench.py --api --node --mof-dir: Hadoop-layout MOF files, the provider front end with the library's
    defaults (it starts the node daemon: HBM store + merge service) and reduce task processes with no
    mapred.uda.* key -- each hosted by the daemon, merging the store's copies of the files in place."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k != "UDA_API_CONF"}
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--api", "--node", "--mof-dir", str(tmp_path), "--reducers",
           "3", "--rows-per-gpu", "3000000", "--maps-per-gpu", "6", "--steps", "1", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["validated"] is True and out["conf_keys"] == 0, out
    t0 = out["task0_stats"]
    assert out["task0_hosted"] and t0["backend"] == "gpu" and t0["device_descriptors"] == 6, t0
    assert t0["host_fetched_bytes"] == 0, t0
    hs = out["provider"]["hbm_store"]
    assert hs["daemon"]["ready"] and hs["loads"] == 6 and hs["merge_service"]["sessions"] >= 9, hs
    assert hs["holders"] == 0, hs  # every hosted task released its descriptors (or its session did)
    assert not os.listdir(tmp_path), "the map outputs are removed after the run"
