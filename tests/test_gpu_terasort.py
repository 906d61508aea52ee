"""GPU end-to-end: TeraSort shuffle+merge on one MI355X (HIP kernels F2/F3/F4 + D2H delivery).

Numerics oracle: the delivered stream is decoded by a J2CQueue-equivalent reader and compared to
a plain Python sort of all generated records (read back from the HBM partition store).
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


@pytest.mark.parametrize("maps,rounds", [(1, 1), (3, 2), (8, 4), (33, 3)])
def test_terasort_stream_matches_python_sort(require_gpu, native, maps, rounds):
    rows = 20000 * maps
    j = _job(rows, maps, rounds, kv_buf_bytes=64 << 10, d2h_piece_bytes=256 << 10)
    reader = J2CQueueReader(max_len=64 << 10)
    j.job.set_python_sink(lambda b: reader.feed(b))
    st = j.step()
    j.check(st)
    assert reader.eof
    # oracle: every generated record, sorted by key (stable on map order)
    recs = []
    for m in range(maps):
        recs += decode_stream(j.job.read_partition(m, 0))
    expect = sorted(recs, key=lambda kv: _text_content(kv[0]))
    assert len(reader.records) == len(expect) == st["records"]
    assert reader.records == expect
    assert st["order_errors"] == 0
    assert st["checksum"] == j.expected_checksum


def test_terasort_repeat_steps_and_device_only(require_gpu):
    j = _job(100000, 5, 3)
    a = j.step()
    b = j.step()
    j.check(a)
    j.check(b)
    assert a["checksum"] == b["checksum"] == j.expected_checksum
    assert a["buffers"] >= a["bytes_in"] // (1 << 20)
    d = _job(100000, 5, 3, deliver_host=False)
    s = d.step()
    d.check(s)
    assert s["buffers"] == 0


def test_merge_tree_many_runs(require_gpu):
    # 300 runs -> 9 merge passes, odd segment counts on several levels
    j = _job(300 * 700, 300, 2)
    st = j.step()
    j.check(st)
    assert st["merge_passes"] == 9


@pytest.mark.parametrize("world,maps,rounds", [
    (2, 3, 3), (3, 2, 4), (4, 1, 1),
    # Known intermittent checksum mismatch (records and order correct) in the 8-thread local-group
    # rehearsal; see docs/BENCHMARKS.md "Known issue". Not the RCCL path bench.py uses.
    pytest.param(8, 2, 16, marks=pytest.mark.xfail(strict=False, reason="intermittent local-group checksum race")),
])
def test_multirank_schedule_local_group(require_gpu, world, maps, rounds):
    """The multi-GPU shuffle schedule (pack -> all-to-all-v rounds -> merge -> deliver) rehearsed
    with `world` ranks sharing one GPU; every reducer must receive exactly its key range."""
    from uda_amd.models.terasort import TeraSortConfig, make_local_group, run_collective
    cfg = TeraSortConfig(rows_per_gpu=12000 * maps, maps_per_rank=maps, rounds=rounds, validate=True,
                         sample_every=64, kv_buf_bytes=64 << 10, d2h_piece_bytes=256 << 10)
    jobs, ck, rec = make_local_group(world, cfg, group=f"t{world}{maps}{rounds}")
    readers = [J2CQueueReader(max_len=64 << 10) for _ in range(world)]
    for j, r in zip(jobs, readers):
        j.set_python_sink(r.feed)
    for step in range(2):
        stats = run_collective(jobs, lambda j: j.run_step())
        for d, st in enumerate(stats):
            assert st["records"] == rec[d]
            assert st["order_errors"] == 0
            assert st["checksum"] == ck[d]
            if world > 1:
                assert st["bytes_sent"] > 0
        if step == 0:
            for d in range(world):
                recs = []
                for j in jobs:  # global map order = (rank, local map)
                    for m in range(maps):
                        recs += decode_stream(j.read_partition(m, d))
                expect = sorted(recs, key=lambda kv: _text_content(kv[0]))
                assert readers[d].records == expect
                readers[d] = J2CQueueReader(max_len=64 << 10)
                jobs[d].set_python_sink(readers[d].feed)


@pytest.mark.parametrize("world", [1, 2])
def test_host_dram_spill_tier(require_gpu, world):
    """Map outputs in pinned host DRAM (jobs larger than HBM): rounds stream H2D, then merge."""
    from uda_amd.models.terasort import TeraSortConfig, make_local_group, run_collective
    cfg = TeraSortConfig(rows_per_gpu=40000, maps_per_rank=4, rounds=3, validate=True, sample_every=64,
                         kv_buf_bytes=64 << 10, d2h_piece_bytes=256 << 10, store="host")
    if world == 1:
        j = _job(40000, 4, 3, store="host", kv_buf_bytes=64 << 10, d2h_piece_bytes=256 << 10)
        reader = J2CQueueReader(max_len=64 << 10)
        j.job.set_python_sink(reader.feed)
        st = j.step()
        j.check(st)
        assert st["bytes_h2d"] == st["bytes_in"]
        recs = []
        for m in range(4):
            recs += decode_stream(j.job.read_partition(m, 0))
        assert reader.records == sorted(recs, key=lambda kv: _text_content(kv[0]))
    else:
        jobs, ck, rec = make_local_group(world, cfg, group="spill2")
        stats = run_collective(jobs, lambda j: j.run_step())
        for d, st in enumerate(stats):
            assert st["records"] == rec[d] and st["order_errors"] == 0 and st["checksum"] == ck[d]
            assert st["bytes_h2d"] > 0


def test_rccl_communicator_selftest(require_gpu, native):
    """The RCCL data plane of the multi-GPU shuffle on one device: ncclUniqueId bootstrap and the
    grouped ncclSend/ncclRecv counts exchange (world 1)."""
    assert native.rccl_selftest(0, 4096) == "rccl:ok"
