"""End-to-end UdaBridge contract over the in-process loopback transport (CPU, no GPU).

Provider (MOFSupplier) and consumer (NetMerger) run in one process, driven through the C ABI the
way the Java plugins drive JNI. Oracle: a plain Python sort of all map-output records of the
partition (ties across maps may come out in any map order, as in the reference, so equal-key groups
are compared as multisets).
"""
import collections
import os

import pytest

from uda_amd.bridge import UdaConsumer, UdaFallback, UdaProvider, run_reduce
from uda_amd.utils import datagen
from uda_amd.utils.ifile import EOF_MARKER, decode_stream
from uda_amd.utils.mof import write_mof


def expected(maps, partition, key_class):
    recs = [kv for m in maps for kv in m[partition]]
    return sorted(recs, key=datagen.sort_key(key_class))


def check_output(got, want, key_class):
    kf = datagen.sort_key(key_class)
    assert [kf(kv) for kv in got] == [kf(kv) for kv in want]
    assert collections.Counter(got) == collections.Counter(want)


@pytest.fixture
def provider(tmp_path):
    p = UdaProvider()
    yield p
    p.close()


def publish(provider, tmp_path, job, maps, codec=None, on_disk=True):
    streams = datagen.streams(maps)
    ids = []
    for i, parts in enumerate(streams):
        mid = f"attempt_{job}_m_{i:06d}_0"
        if on_disk:
            path, _ = write_mof(str(tmp_path), mid, parts, codec=codec)
            provider.add_mof_file(job, mid, path)
        else:
            from uda_amd.utils.mof import encode_partitions
            data, index = encode_partitions(parts, codec)
            provider.add_mof_memory(job, mid, data, index)
        ids.append(mid)
    return ids


@pytest.mark.parametrize("on_disk", [True, False])
def test_wordcount_online(provider, tmp_path, on_disk):
    maps = datagen.wordcount(num_maps=7, reducers=3, words_per_map=3000)
    ids = publish(provider, tmp_path, "job_1_0001", maps, on_disk=on_disk)
    for r in range(3):
        recs, st, c = run_reduce("host-a", "job_1_0001", ids, r, datagen.TEXT)
        check_output(recs, expected(maps, r, datagen.TEXT), datagen.TEXT)
        assert st["maps_fetched"] == 7 and st["finished"]
        assert c.failure is None
        assert c.fetch_over_calls == 1  # fewer than 20 maps: one report at the end


def test_terasort_small_buffers_and_progress(provider, tmp_path):
    maps = datagen.terasort(num_maps=45, reducers=2, rows_per_map=300)
    ids = publish(provider, tmp_path, "job_1_0002", maps)
    # 16 KiB fetch buffers force many chunks per MOF (records straddle chunk boundaries: the join),
    # 64 KiB delivery buffers force many dataFromUda calls
    recs, st, c = run_reduce("h", "job_1_0002", ids, 1, datagen.TEXT, max_buf_kb=16, kv_buf_size=64 << 10)
    check_output(recs, expected(maps, 1, datagen.TEXT), datagen.TEXT)
    assert c.fetch_over_calls == 3   # every 20 maps + the last one (45 = 20 + 20 + 5)
    assert c.buffers > 5


def test_delivery_framing_matches_reference_packing(provider, tmp_path):
    # buffers are packed greedily with whole records (J2CQueueReader asserts no record straddles
    # buffers and no buffer exceeds kv_buf_size); the last buffer ends with the EOF marker
    maps = datagen.secondary_sort(num_maps=5, reducers=1, rows_per_map=400)
    ids = publish(provider, tmp_path, "job_1_0003", maps)
    recs, st, c = run_reduce("h", "job_1_0003", ids, 0, datagen.TEXT, kv_buf_size=8192)
    want = expected(maps, 0, datagen.TEXT)
    check_output(recs, want, datagen.TEXT)
    total = sum(len(datagen.streams([[[kv]]])[0][0]) - 2 for kv in want) + 2
    assert c.bytes == total
    # greedy packing leaves less than one record of slack per buffer
    max_rec = max(len(datagen.streams([[[kv]]])[0][0]) - 2 for kv in want)
    assert c.buffers <= total // (8192 - max_rec) + 1


@pytest.mark.parametrize("codec", ["snappy", "lzo"])
def test_compressed_map_outputs(provider, tmp_path, codec):
    maps = datagen.wordcount(num_maps=6, reducers=2, words_per_map=4000, seed=9)
    ids = publish(provider, tmp_path, "job_1_0004", maps, codec=codec)
    recs, st, c = run_reduce("h", "job_1_0004", ids, 0, datagen.TEXT, codec=codec, max_buf_kb=16)
    check_output(recs, expected(maps, 0, datagen.TEXT), datagen.TEXT)


@pytest.mark.parametrize("ratio", ["0.20", "0.0", "1.0"])
def test_compressed_buffer_split(provider, tmp_path, ratio):
    """reducer.cc:463-491: a compressed job splits each 2 x buffer pair into a fetch side and an
    uncompressed side (codec block + min buffer + ratio of the rest; the fetch side is capped by
    mapred.rdma.buf.size, the excess moving to the uncompressed side)."""
    maps = datagen.wordcount(num_maps=4, reducers=1, words_per_map=3000, seed=5)
    ids = publish(provider, tmp_path, "job_1_0044", maps, codec="snappy")
    conf = {"mapred.rdma.compression.buffer.ratio": ratio, "mapred.rdma.buf.size": 512}
    recs, st, c = run_reduce("h", "job_1_0044", ids, 0, datagen.TEXT, codec="snappy", max_buf_kb=512, conf=conf)
    check_output(recs, expected(maps, 0, datagen.TEXT), datagen.TEXT)
    pair = 2 * 512 * 1024
    hard_min = 256 * 1024 + 16 * 1024
    uncomp = hard_min + int((pair - hard_min - 16 * 1024) * float(ratio))
    fetch = pair - uncomp
    spare = max(0, fetch - 512 * 1024)
    assert (st["fetch_buf_bytes"], st["uncomp_buf_bytes"]) == (fetch - spare, uncomp + spare)
    assert st["fetch_buf_bytes"] + st["uncomp_buf_bytes"] == pair


def test_unsupported_lzo_decompressor_variant_fails(provider, tmp_path):
    maps = datagen.wordcount(num_maps=2, reducers=1, words_per_map=100, seed=5)
    publish(provider, tmp_path, "job_1_0045", maps, codec="lzo")
    with pytest.raises(Exception, match="lzo.decompressor"):
        UdaConsumer(2, "job_1_0045", "attempt_job_1_0045_r_000000_0", datagen.TEXT, codec="lzo",
                    conf={"io.compression.codec.lzo.decompressor": "LZO1F"})


def test_hybrid_merge_spills_lpqs(provider, tmp_path):
    maps = datagen.terasort(num_maps=23, reducers=1, rows_per_map=200, seed=4)
    ids = publish(provider, tmp_path, "job_1_0005", maps)
    d1, d2 = tmp_path / "local1", tmp_path / "local2"
    d1.mkdir()
    d2.mkdir()
    recs, st, c = run_reduce("h", "job_1_0005", ids, 0, datagen.TEXT, approach=2, lpq_size=5,
                             local_dirs=(str(d1), str(d2)))
    check_output(recs, expected(maps, 0, datagen.TEXT), datagen.TEXT)
    assert st["lpqs"] == 5          # 23 maps / lpq 5 -> 4 regular + 1 for the remainder (> 1)
    assert st["spill_bytes"] > 0
    assert not os.listdir(d1) and not os.listdir(d2)  # LPQ files are transient


def test_hybrid_lpq_checkpoint_resume(provider, tmp_path, monkeypatch):
    """mapred.uda.lpq.checkpoint: attempt 0 fails after its 2nd LPQ spill; the LPQ files and the
    manifest survive; attempt 1 of the same partition restores both LPQs, fetches only the other
    MOFs and produces the same merged output; everything is removed after success."""
    maps = datagen.terasort(num_maps=23, reducers=1, rows_per_map=200, seed=4)
    ids = publish(provider, tmp_path, "job_1_0015", maps)
    d1 = tmp_path / "ld"
    d1.mkdir()
    conf = {"mapred.uda.lpq.checkpoint": 1}
    kw = dict(approach=2, lpq_size=5, local_dirs=(str(d1),), conf=conf)
    monkeypatch.setenv("UDA_FAULT_LPQ_DONE", "2")
    c = UdaConsumer(len(ids), "job_1_0015", "attempt_job_1_0015_r_000000_0", datagen.TEXT, **kw)
    for m in ids:
        c.fetch("h", "job_1_0015", m, 0)
    with pytest.raises(UdaFallback, match="injected"):
        c.wait(60)
    c.close()
    monkeypatch.delenv("UDA_FAULT_LPQ_DONE")
    manifest = d1 / "uda.attempt_job_1_0015_r_000000.lpq.manifest"
    lines = manifest.read_text().splitlines()
    assert [ln.split()[1] for ln in lines] == ["0", "1"]
    kept = sorted(os.listdir(d1))
    assert len(kept) == 3  # manifest + 2 LPQ files; the in-progress LPQ was removed
    restored = {m for ln in lines for m in ln.split()[4].split(",")}
    assert len(restored) == 8  # 23 maps / lpq 5: LPQ sizes 4,4,5,5,5 (remainder spread)
    recs, st, _ = run_reduce("h", "job_1_0015", ids, 0, datagen.TEXT, **kw)
    check_output(recs, expected(maps, 0, datagen.TEXT), datagen.TEXT)
    assert st["restored_lpqs"] == 2 and st["restored_maps"] == 8 and st["maps_fetched"] == 23
    assert st["lpqs"] == 3  # only the remaining LPQs were built
    assert not os.listdir(d1)


def test_int_and_bytes_keys(provider, tmp_path):
    import random
    rng = random.Random(8)
    for key_class, mk in [(datagen.INT, lambda: rng.randrange(0, 10**6).to_bytes(4, "big")),
                          (datagen.BYTES, lambda: (lambda s: len(s).to_bytes(4, "big") + s)(
                              bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 12)))))]:
        kf = datagen.sort_key(key_class)
        maps = [[sorted([(mk(), b"v%d" % i) for i in range(300)], key=kf)] for _ in range(4)]
        job = "job_k_%d" % len(key_class)
        ids = publish(provider, tmp_path, job, maps)
        recs, st, c = run_reduce("h", job, ids, 0, key_class)
        check_output(recs, expected(maps, 0, key_class), key_class)


def test_unsupported_key_class_raises_for_fallback(provider):
    with pytest.raises(RuntimeError, match="UdaRuntimeException"):
        UdaConsumer(1, "job_x", "attempt_x_r_0", "org.apache.hadoop.io.DoubleWritable")


def test_unknown_mof_triggers_failure_once(provider, tmp_path):
    c = UdaConsumer(2, "job_missing", "attempt_job_missing_r_000000_0", datagen.TEXT)
    c.fetch("h", "job_missing", "attempt_nope_m_0", 0)
    c.fetch("h", "job_missing", "attempt_nope_m_1", 0)
    with pytest.raises(UdaFallback):
        c.wait(30)
    c.close()
    assert c.failure_calls == 1


def test_injected_fetch_fault(provider, tmp_path, monkeypatch):
    maps = datagen.wordcount(num_maps=4, reducers=1, words_per_map=500)
    ids = publish(provider, tmp_path, "job_1_0006", maps)
    monkeypatch.setenv("UDA_FAULT_FETCH", "3")
    c = UdaConsumer(len(ids), "job_1_0006", "attempt_job_1_0006_r_000000_0", datagen.TEXT, max_buf_kb=16)
    for m in ids:
        c.fetch("h", "job_1_0006", m, 0)
    with pytest.raises(UdaFallback, match="injected"):
        c.wait(30)
    c.close()
    assert c.failure_calls == 1


def test_eof_only_partition(provider, tmp_path):
    ids = publish(provider, tmp_path, "job_1_0007", [[[]], [[]]])
    recs, st, c = run_reduce("h", "job_1_0007", ids, 0, datagen.TEXT)
    assert recs == [] and c.bytes == len(EOF_MARKER)


def test_cpu_merge_binding_matches_python(native):
    maps = datagen.secondary_sort(num_maps=9, reducers=1, rows_per_map=200, seed=12)
    runs = [s[0] for s in datagen.streams(maps)]
    out, lens = native.cpu_merge(runs, datagen.TEXT, 4096)
    assert all(n <= 4096 for n in lens) and out.endswith(EOF_MARKER)
    check_output(decode_stream(out), expected(maps, 0, datagen.TEXT), datagen.TEXT)


def test_injected_aio_fault_fails_once(provider, tmp_path, monkeypatch):
    """A disk read error on the provider (io_uring completion -EIO) surfaces as exactly one
    failureInUda on the consumer (SURVEY §7.4 fault matrix)."""
    maps = datagen.wordcount(num_maps=3, reducers=1, words_per_map=2000, seed=21)
    ids = publish(provider, tmp_path, "job_1_0008", maps, on_disk=True)
    monkeypatch.setenv("UDA_FAULT_AIO", "2")
    c = UdaConsumer(len(ids), "job_1_0008", "attempt_job_1_0008_r_000000_0", datagen.TEXT, max_buf_kb=16)
    for m in ids:
        c.fetch("h", "job_1_0008", m, 0)
    with pytest.raises(UdaFallback):
        c.wait(30)
    c.close()
    assert c.failure_calls == 1


def test_injected_host_alloc_fault_raises_on_init(monkeypatch):
    monkeypatch.setenv("UDA_FAULT_HOST_ALLOC", "1")
    with pytest.raises(RuntimeError, match="UdaRuntimeException"):
        UdaConsumer(2, "job_1_0009", "attempt_job_1_0009_r_000000_0", datagen.TEXT)


def test_checkpoint_resume_refuses_reexecuted_map(provider, tmp_path, monkeypatch):
    """A map re-executed between reduce attempts (new attempt id) must not be merged next to the
    restored LPQ that holds its old attempt: the checkpoint is discarded and the attempt fails over
    (fallback), and a clean attempt then produces the right output."""
    maps = datagen.terasort(num_maps=23, reducers=1, rows_per_map=200, seed=4)
    ids = publish(provider, tmp_path, "job_1_0016", maps)
    d1 = tmp_path / "ld"
    d1.mkdir()
    kw = dict(approach=2, lpq_size=5, local_dirs=(str(d1),), conf={"mapred.uda.lpq.checkpoint": 1})
    monkeypatch.setenv("UDA_FAULT_LPQ_DONE", "2")
    c = UdaConsumer(len(ids), "job_1_0016", "attempt_job_1_0016_r_000000_0", datagen.TEXT, **kw)
    for m in ids:
        c.fetch("h", "job_1_0016", m, 0)
    with pytest.raises(UdaFallback, match="injected"):
        c.wait(60)
    c.close()
    monkeypatch.delenv("UDA_FAULT_LPQ_DONE")
    manifest = d1 / "uda.attempt_job_1_0016_r_000000.lpq.manifest"
    restored = sorted({m for ln in manifest.read_text().splitlines() for m in ln.split()[4].split(",")})
    # map attempt _0 of one restored task is re-executed as attempt _1 (same data)
    old = restored[0]
    new = old[:-1] + "1"
    mof = maps[ids.index(old)]
    from uda_amd.utils.mof import write_mof
    path, _ = write_mof(str(tmp_path), new, datagen.streams([mof])[0])
    provider.add_mof_file("job_1_0016", new, path)
    ids2 = [new if m == old else m for m in ids]
    c = UdaConsumer(len(ids2), "job_1_0016", "attempt_job_1_0016_r_000000_1", datagen.TEXT, **kw)
    with pytest.raises(Exception, match="re-executed"):
        for m in ids2:
            c.fetch("h", "job_1_0016", m, 0)
    c.close()
    assert not os.listdir(d1)  # manifest and restored LPQ files are gone
    recs, st, _ = run_reduce("h", "job_1_0016", ids2, 0, datagen.TEXT, **kw)
    check_output(recs, expected(maps, 0, datagen.TEXT), datagen.TEXT)
    assert st["restored_lpqs"] == 0 and st["maps_fetched"] == 23


def test_checkpoint_and_spills_never_follow_planted_links(provider, tmp_path):
    """A reduce task's local dirs may be writable by another user (YARN's usercache/<user>/appcache): a
    checkpoint manifest that is a symlink (or somebody else's file) is not trusted, and LPQ spill files are
    created fresh, never through a link planted at their names. The files the links point to survive
    unchanged and the task still merges correctly."""
    maps = datagen.terasort(num_maps=23, reducers=1, rows_per_map=200, seed=7)
    job = "job_1_0017"
    ids = publish(provider, tmp_path, job, maps)
    d1 = tmp_path / "ld"
    d1.mkdir()
    victim = tmp_path / "victim.bin"
    victim.write_bytes(b"precious" * 100)
    fake_lpq = tmp_path / "fake.lpq"
    fake_lpq.write_bytes(b"x" * 64)
    # a manifest (outside the dir, linked in) naming a file the task would read back and unlink
    real_manifest = tmp_path / "planted.manifest"
    real_manifest.write_text(f"lpq 0 64 {fake_lpq} {','.join(ids[:4])}\n")
    os.symlink(real_manifest, d1 / f"uda.attempt_{job}_r_000000.lpq.manifest")
    for i in range(5):  # every LPQ spill name of the attempt points at the victim
        os.symlink(victim, d1 / f"uda.attempt_{job}_r_000000_0.lpq-{i:03d}")
    kw = dict(approach=2, lpq_size=5, local_dirs=(str(d1),), conf={"mapred.uda.lpq.checkpoint": 1})
    recs, st, _ = run_reduce("h", job, ids, 0, datagen.TEXT, **kw)
    check_output(recs, expected(maps, 0, datagen.TEXT), datagen.TEXT)
    assert st["restored_lpqs"] == 0 and st["maps_fetched"] == 23
    assert victim.read_bytes() == b"precious" * 100
    assert fake_lpq.exists() and fake_lpq.read_bytes() == b"x" * 64
    assert real_manifest.read_text().startswith("lpq 0 64")
