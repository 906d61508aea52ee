"""GPU end-to-end: TeraSort shuffle+merge on one MI355X (HIP kernels F2/F3/F4 + SDMA delivery).

Numerics oracle: the delivered stream of every reducer is decoded by a J2CQueue-equivalent reader
and compared to a plain Python sort of all generated records (read back from the partition store).
"""
import pytest

from uda_amd.parallel.dist import DistContext
from uda_amd.utils.ifile import J2CQueueReader, decode_stream

pytestmark = pytest.mark.gpu


def _job(rows, maps, rounds, validate=True, **kw):
    from uda_amd.models.terasort import TeraSortConfig, TeraSortShuffle
    cfg = TeraSortConfig(rows_per_gpu=rows, maps_per_rank=maps, rounds=rounds, validate=validate,
                         sample_every=64, **kw)
    j = TeraSortShuffle(DistContext(), cfg, device=0)
    j.setup()
    return j


def _text_content(key: bytes) -> bytes:
    return key[1:]  # Text VInt(10) prefix


def _sorted_all(parts):
    recs = []
    for p in parts:
        recs += decode_stream(p)
    return sorted(recs, key=lambda kv: _text_content(kv[0]))


SMALL = dict(kv_buf_bytes=64 << 10, d2h_piece_bytes=256 << 10)


@pytest.mark.parametrize("maps,rounds,reducers", [(1, 1, 1), (3, 2, 1), (8, 4, 1), (33, 3, 1), (5, 3, 4), (4, 1, 3)])
def test_terasort_stream_matches_python_sort(require_gpu, native, maps, rounds, reducers):
    rows = 20000 * maps
    j = _job(rows, maps, rounds, reducers=reducers, **SMALL)
    readers = [J2CQueueReader(max_len=64 << 10) for _ in range(reducers)]
    j.use_python_sink(lambda r, b: readers[r].feed(b), with_reducer=True)
    st = j.step()
    j.check(st)
    assert all(r.eof for r in readers)
    # oracle: every generated record, sorted by key; reducer outputs concatenate to the total order
    expect = _sorted_all(j.job.read_partition(m, 0) for m in range(maps))
    got = [kv for r in readers for kv in r.records]
    assert len(got) == len(expect) == st["records"]
    assert got == expect
    assert [len(r.records) for r in readers] == list(j.job.reducer_records())
    assert st["order_errors"] == 0
    assert st["checksum"] == j.expected_checksum


def test_terasort_repeat_steps_j2c_sink_and_device_only(require_gpu):
    j = _job(100000, 5, 3, reducers=2)
    a = j.step()
    b = j.step()
    j.check(a)  # includes the native J2C consumer's record counts, framing and EOF per reducer
    j.check(b)
    assert a["checksum"] == b["checksum"] == j.expected_checksum
    assert sum(a["consumer_records"]) == a["records"]
    assert a["buffers"] >= a["bytes_in"] // (1 << 20)
    c = j.step(validate=False)
    j.check(c)
    assert not c["validated"]
    d = _job(100000, 5, 3, deliver_host=False)
    s = d.step()
    d.check(s)
    assert s["buffers"] == 0


@pytest.mark.parametrize("mode", ["sdma", "hip"])
def test_delivery_modes(require_gpu, mode):
    """Both delivery copy paths (explicit SDMA engines / hipMemcpyAsync) deliver the same stream."""
    j = _job(60000, 3, 2, reducers=2, d2h=mode, d2h_engines=2, **SMALL)
    st = j.step()
    j.check(st)
    name = j.job.delivery_name
    assert name.startswith(mode)


def test_merge_tree_many_runs(require_gpu):
    # 300 runs -> 9 merge passes, odd segment counts on several levels
    j = _job(300 * 700, 300, 2)
    st = j.step()
    j.check(st)
    assert st["merge_passes"] == 9


@pytest.mark.parametrize("world,maps,rounds,reducers,map_sort", [
    (2, 3, 3, 1, False), (3, 2, 4, 1, False), (4, 1, 1, 1, False), (8, 2, 16, 1, False), (4, 3, 4, 3, False),
    (8, 2, 4, 2, False), (4, 3, 4, 3, True), (8, 2, 16, 2, True),
])
def test_multirank_schedule_local_group(require_gpu, world, maps, rounds, reducers, map_sort):
    """The multi-GPU shuffle schedule (cell split -> all-to-all-v rounds -> grouped merge ->
    deliver) rehearsed with `world` ranks sharing one GPU; every reducer must receive exactly its
    key range, and every received slice must hash to what its sender computed. map_sort: the map
    outputs come from the device radix sort of unsorted map input (the bench default)."""
    from uda_amd.models.terasort import TeraSortConfig, check_stats, make_local_group, run_collective
    cfg = TeraSortConfig(rows_per_gpu=12000 * maps, maps_per_rank=maps, rounds=rounds, reducers=reducers,
                         validate=True, sample_every=64, map_sort=map_sort, **SMALL)
    jobs, ck, rec = make_local_group(world, cfg, group=f"t{world}{maps}{rounds}{reducers}{int(map_sort)}")
    readers = [[J2CQueueReader(max_len=64 << 10) for _ in range(reducers)] for _ in range(world)]

    def attach(d):
        jobs[d].set_python_sink(lambda r, b: readers[d][r].feed(b), True)

    for d in range(world):
        attach(d)
    for step in range(2):
        stats = run_collective(jobs, lambda j: j.run_step(True))
        for d, st in enumerate(stats):
            check_stats(st, rec[d], ck[d], jobs[d].reducer_records())
            assert st["exchange_errors"] == 0
            if world > 1:
                assert st["bytes_sent"] > 0
        if step == 0:
            for d in range(world):
                expect = _sorted_all(j.read_partition(m, d) for j in jobs for m in range(maps))
                got = [kv for r in readers[d] for kv in r.records]
                assert got == expect
                readers[d] = [J2CQueueReader(max_len=64 << 10) for _ in range(reducers)]
                attach(d)


@pytest.mark.parametrize("world", [1, 2])
def test_host_dram_spill_tier(require_gpu, world):
    """Map outputs in pinned host DRAM (jobs larger than HBM): rounds stream H2D, then merge."""
    from uda_amd.models.terasort import TeraSortConfig, check_stats, make_local_group, run_collective
    cfg = TeraSortConfig(rows_per_gpu=40000, maps_per_rank=4, rounds=3, reducers=2, validate=True, sample_every=64,
                         store="host", **SMALL)
    if world == 1:
        j = _job(40000, 4, 3, store="host", reducers=2, **SMALL)
        readers = [J2CQueueReader(max_len=64 << 10) for _ in range(2)]
        j.use_python_sink(lambda r, b: readers[r].feed(b), with_reducer=True)
        st = j.step()
        j.check(st)
        assert st["bytes_h2d"] == st["bytes_in"]
        got = [kv for r in readers for kv in r.records]
        assert got == _sorted_all(j.job.read_partition(m, 0) for m in range(4))
    else:
        jobs, ck, rec = make_local_group(world, cfg, group="spill2")
        sinks = []
        for j in jobs:
            from uda_amd import native
            s = native().J2CSink(2, cfg.kv_buf_bytes)
            j.set_j2c_sink(s)
            sinks.append(s)
        stats = run_collective(jobs, lambda j: j.run_step(True))
        for d, st in enumerate(stats):
            check_stats(st, rec[d], ck[d], jobs[d].reducer_records())
            assert [sinks[d].records(i) for i in range(2)] == list(jobs[d].reducer_records())
            assert st["bytes_h2d"] > 0


def test_rccl_communicator_selftest(require_gpu, native):
    """The RCCL data plane of the multi-GPU shuffle on one device: ncclUniqueId bootstrap and the
    grouped ncclSend/ncclRecv counts exchange (world 1)."""
    assert native.rccl_selftest(0, 4096) == "rccl:ok"


@pytest.mark.parametrize("reducers,rounds", [(1, 3), (3, 2)])
def test_disk_store_tier(require_gpu, tmp_path, reducers, rounds):
    """Map outputs as MOF files on local disks (the tier for jobs larger than HBM + DRAM): each
    round's cells are read with io_uring O_DIRECT into a pinned chunk ring and copied to HBM."""
    d1, d2 = tmp_path / "d1", tmp_path / "d2"
    d1.mkdir()
    d2.mkdir()
    j = _job(30000, 5, rounds, store="disk", local_dirs=f"{d1},{d2}", reducers=reducers, **SMALL)
    assert j.job.store_name.startswith("disk[")
    assert len(list(d1.iterdir())) == 3 and len(list(d2.iterdir())) == 2  # MOF files striped
    readers = [J2CQueueReader(max_len=64 << 10) for _ in range(reducers)]
    j.use_python_sink(lambda r, b: readers[r].feed(b), with_reducer=True)
    st = j.step()
    j.check(st)
    assert st["bytes_h2d"] == st["bytes_in"]
    got = [kv for r in readers for kv in r.records]
    assert got == _sorted_all(j.job.read_partition(m, 0) for m in range(5))
    del j
    import gc
    gc.collect()
    assert not list(d1.iterdir()) and not list(d2.iterdir())  # files removed with the store


@pytest.mark.parametrize("world,store,h2d_sdma", [(2, "disk", "1"), (3, "disk", "1"), (3, "host", "1"),
                                                 (3, "host", "0")])
def test_spill_tiers_multirank_staged(require_gpu, tmp_path, monkeypatch, world, store, h2d_sdma):
    """Spill tiers at world > 1: every round's outgoing slices are staged into HBM (double-buffered
    send staging, one message per peer) and every peer pulls them with the strict pairing and
    device-memory checks of the exchange; staging runs on the staging thread (SDMA / io_uring) or,
    with UDA_H2D_SDMA=0, as a copy kernel on the comm stream. Two steps reuse both staging parities."""
    from uda_amd.models.terasort import TeraSortConfig, check_stats, make_local_group, run_collective
    monkeypatch.setenv("UDA_H2D_SDMA", h2d_sdma)
    cfg = TeraSortConfig(rows_per_gpu=30000, maps_per_rank=3, rounds=5, reducers=2, validate=True, sample_every=64,
                         store=store, local_dirs=str(tmp_path), **SMALL)
    jobs, ck, rec = make_local_group(world, cfg, group=f"spill{world}{store}{h2d_sdma}")
    readers = [[J2CQueueReader(max_len=64 << 10) for _ in range(2)] for _ in range(world)]
    for d in range(world):
        jobs[d].set_python_sink(lambda r, b, d=d: readers[d][r].feed(b), True)
    for step in range(2):
        stats = run_collective(jobs, lambda j: j.run_step(True))
        for d, st in enumerate(stats):
            check_stats(st, rec[d], ck[d], jobs[d].reducer_records())
            assert st["exchange_errors"] == 0
            assert st["bytes_sent"] > 0 and st["bytes_h2d"] >= st["bytes_sent"]
        if step == 0:
            for d in range(world):
                expect = _sorted_all(j.read_partition(m, d) for j in jobs for m in range(3))
                assert [kv for r in readers[d] for kv in r.records] == expect
                readers[d] = [J2CQueueReader(max_len=64 << 10) for _ in range(2)]
                jobs[d].set_python_sink(lambda r, b, d=d: readers[d][r].feed(b), True)


@pytest.mark.parametrize("world,maps,rounds,reducers,map_sort", [(8, 2, 16, 1, False), (4, 3, 4, 3, True),
                                                                  (1, 6, 2, 2, False)])
def test_no_kernel_writes_past_its_buffers(require_gpu, monkeypatch, world, maps, rounds, reducers, map_sort):
    """UDA_DEVICE_GUARD=1 puts a guard tail behind every device buffer and checks it at free: the map
    sort, exchange, K-way plan + merge, validation and delivery of a multi-rank schedule (8 ranks on one
    GPU, 16 rounds, as in a one-off checksum mismatch of that case) leave every tail intact."""
    import gc

    from uda_amd import native
    from uda_amd.models.terasort import TeraSortConfig, check_stats, make_local_group, run_collective
    monkeypatch.setenv("UDA_DEVICE_GUARD", "1")
    before = native().device_guard_violations()
    cfg = TeraSortConfig(rows_per_gpu=12000 * maps, maps_per_rank=maps, rounds=rounds, reducers=reducers,
                         validate=True, sample_every=64, map_sort=map_sort, **SMALL)
    jobs, ck, rec = make_local_group(world, cfg, group=f"guard{world}{maps}{rounds}{reducers}")
    for _ in range(2):
        readers = [[J2CQueueReader(max_len=64 << 10) for _ in range(reducers)] for _ in range(world)]
        for d in range(world):
            jobs[d].set_python_sink(lambda r, b, d=d, rd=readers: rd[d][r].feed(b), True)
        stats = run_collective(jobs, lambda j: j.run_step(True))
        for d, st in enumerate(stats):
            check_stats(st, rec[d], ck[d], jobs[d].reducer_records())
    del jobs, stats
    gc.collect()
    assert native().device_guard_violations() == before


@pytest.mark.parametrize("env", [{"UDA_KWAY": "0"}, {"UDA_KWAY_TARGET": "5000"}, {"UDA_KWAY_CAP": "1536"},
                                 {"UDA_KWAY_FILL": "85", "UDA_KWAY_CAP": "512"}, {"UDA_KWAY_CAP": "1024"},
                                 {"UDA_KWAY_STAGED": "1"}, {"UDA_KWAY_STAGED": "1", "UDA_KWAY_CAP": "512"},
                                 {"UDA_KWAY_STAGED": "1", "UDA_KWAY_TARGET": "5000"}])
def test_kway_merge_matches_pairwise_tree(require_gpu, monkeypatch, env):
    """The single-pass K-way merge (default) and the pairwise merge-path tree (UDA_KWAY=0) order
    records identically; UDA_KWAY_TARGET above the LDS capacity routes every cell through the
    wave-level priority queue, which must give the same stream; so must every cell capacity."""
    ref = _job(60000, 6, 2, reducers=2, **SMALL)
    readers = [J2CQueueReader(max_len=64 << 10) for _ in range(2)]
    ref.use_python_sink(lambda r, b: readers[r].feed(b), with_reducer=True)
    st = ref.step()
    ref.check(st)
    assert st["merge_passes"] == 1  # single pass
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    alt = _job(60000, 6, 2, reducers=2, **SMALL)
    readers2 = [J2CQueueReader(max_len=64 << 10) for _ in range(2)]
    alt.use_python_sink(lambda r, b: readers2[r].feed(b), with_reducer=True)
    st2 = alt.step()
    alt.check(st2)
    assert [r.records for r in readers2] == [r.records for r in readers]
    if "UDA_KWAY" in env:
        assert st2["merge_passes"] == 3  # ceil(log2(6)) pairwise passes


@pytest.mark.parametrize("env", [{}, {"UDA_KWAY_TARGET": "100000"}, {"UDA_KWAY_CAP": "1792"}, {"UDA_KWAY_STAGED": "1"}])
def test_kway_many_runs_per_group(require_gpu, monkeypatch, env):
    """200 runs per group (an 8-GPU round has 8 x 32 = 256): the single-pass merge sizes its per-slice
    LDS tables by the plan's largest group and must order records like the pairwise tree, on the LDS
    path, on the wave-PQ path (UDA_KWAY_TARGET above the capacity) and at the 1792-record capacity."""
    ref_env = {"UDA_KWAY": "0"}
    out = []
    for e in (ref_env, env):
        for k in ("UDA_KWAY", "UDA_KWAY_TARGET", "UDA_KWAY_CAP", "UDA_KWAY_STAGED"):
            monkeypatch.delenv(k, raising=False)
        for k, v in e.items():
            monkeypatch.setenv(k, v)
        j = _job(200 * 300, 200, 2, reducers=2, **SMALL)
        readers = [J2CQueueReader(max_len=64 << 10) for _ in range(2)]
        j.use_python_sink(lambda r, b, rd=readers: rd[r].feed(b), with_reducer=True)
        st = j.step()
        j.check(st)
        out.append([r.records for r in readers])
        assert st["merge_passes"] == (8 if e is ref_env else 1)
    assert out[0] == out[1]


@pytest.mark.parametrize("world,store", [(1, "hbm"), (1, "host"), (2, "hbm")])
def test_replan_every_step(require_gpu, world, store):
    """replan=True: each step recomputes the cell splits from the map outputs (and, for world>1,
    re-exchanges the slice counts) inside the timed step; unchanged outputs must reproduce the plan."""
    from uda_amd.models.terasort import TeraSortConfig, check_stats, make_local_group, run_collective
    cfg = TeraSortConfig(rows_per_gpu=40000, maps_per_rank=3, rounds=3, reducers=2, validate=True, sample_every=64,
                         store=store, replan=True, **SMALL)
    jobs, ck, rec = make_local_group(world, cfg, group=f"replan{world}{store}")
    for _ in range(2):
        stats = run_collective(jobs, lambda j: j.run_step(True))
        for d, st in enumerate(stats):
            check_stats(st, rec[d], ck[d], jobs[d].reducer_records())
            assert st["plan_ms"] > 0


def test_multirank_schedule_beside_busy_streams(require_gpu, native):
    """Regression for the r5 multi-rank "checksum mismatch" (records, order and every slice correct): the
    generation checksums were zeroed by a null-stream hipMemset, which the generation kernels on a
    non-blocking stream did not wait for. Other streams of the process kept busy with device copies
    (`start_gpu_noise`, the same queue pressure the per-device stream pool added) made it fail every group
    after the first; now every fresh group plans (its generation checksums match the store: plan()
    checks) and validates."""
    from uda_amd.models.terasort import TeraSortConfig, check_stats, make_local_group, run_collective
    native.start_gpu_noise(0, 8, 8 << 20)
    try:
        for g in range(4):
            cfg = TeraSortConfig(rows_per_gpu=24000, maps_per_rank=2, rounds=16, reducers=1, validate=True,
                                 sample_every=64, kv_buf_bytes=64 << 10, d2h_piece_bytes=256 << 10)
            jobs, ck, rec = make_local_group(8, cfg, group=f"busy{g}")
            stats = run_collective(jobs, lambda j: j.run_step(True))
            for d, st in enumerate(stats):
                check_stats(st, rec[d], ck[d], jobs[d].reducer_records())
            del jobs
    finally:
        assert native.stop_gpu_noise() > 0
