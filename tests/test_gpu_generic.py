"""GPU generic merge (F1 record index, F2 normalize + full-key tie-break, F3 merge tree, F4 scan +
gather) against the CPU reference heap merge: the merged streams must be byte-identical (both
break key ties by run order, then position)."""
import os
import random

import pytest

from uda_amd import ops
from uda_amd.bridge import UdaProvider, run_reduce
from uda_amd.utils import datagen
from uda_amd.utils.ifile import J2CQueueReader, encode_stream, text

pytestmark = pytest.mark.gpu


def _cases():
    yield "wordcount", datagen.TEXT, [s[0] for s in datagen.streams(datagen.wordcount(9, 1, 4000))]
    yield "secondary", datagen.TEXT, [s[0] for s in datagen.streams(datagen.secondary_sort(17, 1, 700))]
    yield "terasort", datagen.TEXT, [s[0] for s in datagen.streams(datagen.terasort(5, 1, 500))]
    rng = random.Random(4)
    ints = [encode_stream(sorted([(rng.randrange(0, 50).to_bytes(4, "big"), b"v%d" % i) for i in range(400)]))
            for _ in range(6)]
    yield "int-dups", datagen.INT, ints
    bw = lambda s: len(s).to_bytes(4, "big") + s  # noqa: E731
    byt = [encode_stream(sorted([(bw(bytes(rng.getrandbits(2) for _ in range(rng.randint(0, 20)))), b"")
                                 for _ in range(300)], key=lambda kv: kv[0][4:])) for _ in range(5)]
    yield "bytes", datagen.BYTES, byt
    # long common prefixes: ties on the 8-byte prefix must be settled on the full key
    pref = b"0123456789abcdef-common-prefix-"
    keys = [[text(pref + bytes([rng.randrange(97, 100)]) * rng.randint(0, 3)) for _ in range(200)] for _ in range(4)]
    yield "long-prefix", datagen.TEXT, [encode_stream(sorted([(k, b"x") for k in ks], key=lambda kv: kv[0][1:]))
                                        for ks in keys]
    # values longer than the parallel F1 entry table: those runs take the serial index walk
    big = [encode_stream(sorted([(text(b"k%05d" % rng.randrange(10**5)), os.urandom(rng.randint(200, 3000)))
                                 for _ in range(150)])) for _ in range(3)]
    yield "long-values", datagen.TEXT, big
    mixed = [encode_stream(sorted([(text(b"m%05d" % rng.randrange(10**5)),
                                    os.urandom(rng.randint(600, 900) if rng.random() < 0.02 else rng.randint(0, 40)))
                                   for _ in range(5000)]))] + \
        [s[0] for s in datagen.streams(datagen.wordcount(2, 1, 3000, seed=8))]
    yield "mixed-long", datagen.TEXT, mixed
    yield "empty-runs", datagen.TEXT, [encode_stream([]), encode_stream([(text(b"a"), b"1")]), encode_stream([])]


@pytest.mark.parametrize("name,key_class,runs", list(_cases()), ids=[c[0] for c in _cases()])
def test_gpu_merge_matches_cpu(require_gpu, name, key_class, runs):
    g_body, g_cuts = ops.merge_runs(runs, key_class, "gpu", kv_buf=4096)
    c_body, _ = ops.merge_runs(runs, key_class, "cpu", kv_buf=4096)
    assert g_body == c_body
    r = J2CQueueReader(max_len=4096)
    for b in ops.buffers(g_body, g_cuts):
        r.feed(b)
    assert r.eof


def test_gpu_merge_many_runs(require_gpu):
    runs = [s[0] for s in datagen.streams(datagen.secondary_sort(300, 1, 60, seed=21))]
    g, _ = ops.merge_runs(runs, datagen.TEXT, "gpu")
    c, _ = ops.merge_runs(runs, datagen.TEXT, "cpu")
    assert g == c


def test_gpu_merge_large_runs_parallel_index(require_gpu, native):
    """Runs spanning many F1 superchunks (256 KiB): the parallel index must be used (no serial
    fallback) and match the CPU merge byte for byte."""
    runs = [r[0] for r in native.generate_runs("secondary", 6, 1, 12000, 77)]
    assert min(len(r) for r in runs) > 3 * 256 * 1024
    g, _ = ops.merge_runs(runs, datagen.TEXT, "gpu")
    assert ops.last_stats["f1_serial_runs"] == 0
    c, _ = ops.merge_runs(runs, datagen.TEXT, "cpu")
    assert g == c


def test_gpu_merge_serial_fallback_counted(require_gpu):
    rng = random.Random(5)
    big = [encode_stream(sorted([(text(b"%06d" % rng.randrange(10**6)), os.urandom(1000)) for _ in range(400)]))
           for _ in range(2)]
    small = [s[0] for s in datagen.streams(datagen.wordcount(3, 1, 2000, seed=9))]
    g, _ = ops.merge_runs(big + small, datagen.TEXT, "gpu")
    assert ops.last_stats["f1_serial_runs"] == 2
    c, _ = ops.merge_runs(big + small, datagen.TEXT, "cpu")
    assert g == c


def test_gpu_merge_misframed_text_keys_fall_back(require_gpu):
    """The parallel F1 walk ends chains whose key does not start with its Text length (that is how
    it drops chains entered at non-record bytes). Keys declared Text but not framed as Text (raw
    bytes) must then take the serial index walk and still merge exactly like the CPU."""
    rng = random.Random(11)
    raw = [encode_stream(sorted([(bytes(rng.randrange(200, 256) for _ in range(rng.randint(3, 12))), b"v" * 30)
                                 for _ in range(3000)], key=lambda kv: kv[0][1:]))
           for _ in range(3)]
    good = [s[0] for s in datagen.streams(datagen.secondary_sort(4, 1, 3000, seed=3))]
    g, _ = ops.merge_runs(raw + good, datagen.TEXT, "gpu")
    assert ops.last_stats["f1_serial_runs"] == 3
    c, _ = ops.merge_runs(raw + good, datagen.TEXT, "cpu")
    assert g == c


def test_consumer_gpu_backend(require_gpu, tmp_path):
    from uda_amd.utils.mof import write_mof
    p = UdaProvider()
    try:
        maps = datagen.secondary_sort(num_maps=12, reducers=2, rows_per_map=500, seed=5)
        ids = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_g_m_{i:06d}_0"
            path, _ = write_mof(str(tmp_path), mid, parts, codec="snappy")
            p.add_mof_file("job_g", mid, path)
            ids.append(mid)
        recs_gpu, st, c = run_reduce("h", "job_g", ids, 1, datagen.TEXT, codec="snappy",
                                     conf={"mapred.uda.merge.backend": "gpu"}, kv_buf_size=8192)
        recs_cpu, _, _ = run_reduce("h", "job_g", ids, 1, datagen.TEXT, codec="snappy", kv_buf_size=8192)
        assert st["backend"] == "gpu"
        assert [k for k, _ in recs_gpu] == [k for k, _ in recs_cpu]
        assert sorted(recs_gpu) == sorted(recs_cpu)
    finally:
        p.close()


@pytest.mark.parametrize("drains,step", [(0, 0), (1, 0), (3, 0), (3, 40_000), (0, 20_000)])
def test_consumer_gpu_fetch_drains_and_piecewise_staging(require_gpu, drains, step):
    """Uncompressed in-memory MOFs fetched in 16 KiB requests: the GPU backend's drain-thread count
    and piecewise early H2D staging (landed prefixes copied to HBM while the rest is in flight)
    must deliver exactly the CPU merge's stream."""
    from uda_amd.utils.mof import encode_partitions
    p = UdaProvider()
    try:
        maps = datagen.secondary_sort(num_maps=9, reducers=2, rows_per_map=1500, seed=11)
        ids = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_d_m_{i:06d}_0"
            data, index = encode_partitions(parts)
            p.add_mof_memory("job_d", mid, data, index)
            ids.append(mid)
        conf = {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.fetch.drains": drains,
                "mapred.uda.gpu.early.h2d.step": step}
        recs_gpu, st, _ = run_reduce("h", "job_d", ids, 0, datagen.TEXT, conf=conf, max_buf_kb=16, min_buf_kb=16,
                                     kv_buf_size=8192)
        recs_cpu, _, _ = run_reduce("h", "job_d", ids, 0, datagen.TEXT, max_buf_kb=16, min_buf_kb=16,
                                    kv_buf_size=8192)
        assert st["backend"] == "gpu"
        assert [k for k, _ in recs_gpu] == [k for k, _ in recs_cpu]  # equal keys may come in any run order
        assert sorted(recs_gpu) == sorted(recs_cpu)
    finally:
        p.close()


@pytest.mark.parametrize("phases,drains,maps,kind", [(2, 3, 9, "text"), (3, 1, 9, "text"), (7, 3, 9, "text"),
                                                     (4, 8, 20, "bytes"), (5, 3, 3, "text"), (None, 3, 9, "text")])
def test_consumer_gpu_progressive_phases(require_gpu, phases, drains, maps, kind):
    """mapred.uda.gpu.progressive.phases: partitions fetched in byte phases (all partitions' phase p
    first), each phase's key range below the least last-landed key merged and delivered while later
    phases arrive. The stream must equal the CPU merge's, with records cut by a phase end (partial F1)
    carried into the next phase, and partitions of very different sizes (skewed reducers)."""
    from uda_amd.utils.mof import encode_partitions
    p = UdaProvider()
    try:
        if kind == "text":
            mp = datagen.secondary_sort(num_maps=maps, reducers=2, rows_per_map=1500, seed=13 + (phases or 0))
            key_class = datagen.TEXT
        else:
            mp = datagen.bytes_writable(num_maps=maps, reducers=2, rows_per_map=900, seed=3)
            key_class = datagen.BYTES
        ids = []
        for i, parts in enumerate(datagen.streams(mp)):
            mid = f"attempt_p_m_{i:06d}_0"
            data, index = encode_partitions(parts)
            p.add_mof_memory("job_p", mid, data, index)
            ids.append(mid)
        conf = {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.fetch.drains": drains}
        if phases is not None:  # None: the default, progressive when the task is alone on its device
            conf["mapred.uda.gpu.progressive.phases"] = phases
        recs_gpu, st, _ = run_reduce("h", "job_p", ids, 0, key_class, conf=conf, max_buf_kb=16, min_buf_kb=16,
                                     kv_buf_size=8192)
        recs_cpu, _, _ = run_reduce("h", "job_p", ids, 0, key_class, max_buf_kb=16, min_buf_kb=16, kv_buf_size=8192)
        assert st["backend"] == "gpu" and st["maps_fetched"] == maps
        assert [k for k, _ in recs_gpu] == [k for k, _ in recs_cpu]
        assert sorted(recs_gpu) == sorted(recs_cpu)
        assert st["rpq_rounds"] >= 1  # at least one phase merged before the last one
    finally:
        p.close()


@pytest.mark.parametrize("tier,codec,direct", [("host", None, 1), ("host", None, 0), ("disk", None, 1),
                                               ("disk", "snappy", 1)])
def test_consumer_gpu_hybrid_lpq_rpq(require_gpu, tmp_path, tier, codec, direct):
    """Reduce input larger than the device budget: LPQ merges on the GPU spill to host DRAM or to
    the local dirs (AsyncIO), then RPQ key-range rounds merge the spilled runs on the GPU. On the
    DRAM tier the default is the direct RPQ: no LPQ level, the rounds merge slices of the fetched
    partitions where the fetch put them (mapred.uda.gpu.hybrid.direct=0 keeps the LPQ level)."""
    from uda_amd.utils.mof import write_mof
    p = UdaProvider()
    try:
        maps = datagen.secondary_sort(num_maps=12, reducers=2, rows_per_map=2000, seed=6)
        ids = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_h{tier}{codec}_m_{i:06d}_0"
            path, _ = write_mof(str(tmp_path), mid, parts, codec=codec)
            p.add_mof_file(f"job_h{tier}{codec}", mid, path)
            ids.append(mid)
        d1 = tmp_path / "ld1"
        d1.mkdir()
        conf = {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.merge.bytes": 300_000,
                "mapred.uda.gpu.spill": tier, "mapred.uda.gpu.hybrid.direct": direct}
        recs, st, c = run_reduce("h", f"job_h{tier}{codec}", ids, 0, datagen.TEXT, codec=codec, conf=conf,
                                 kv_buf_size=8192, local_dirs=(str(d1),))
        if tier == "host" and direct:
            assert st["hybrid_direct"] == 1 and st["lpqs"] == 0 and st["rpq_rounds"] >= 3, st
        else:
            assert st["hybrid_direct"] == 0 and st["lpqs"] >= 4 and st["rpq_rounds"] >= 3, st
        want = sorted((kv for m in maps for kv in m[0]), key=datagen.sort_key(datagen.TEXT))
        kf = datagen.sort_key(datagen.TEXT)
        assert [kf(kv) for kv in recs] == [kf(kv) for kv in want]
        assert sorted(recs) == sorted(want)
        assert not os.listdir(d1)  # spill files are transient
    finally:
        p.close()


@pytest.mark.parametrize("workload,phases", [("secondary", 8), ("secondary", 2), ("secondary", 64), ("wordcount", 8),
                                            ("secondary", 0)])
def test_consumer_gpu_progressive_direct_rpq(require_gpu, tmp_path, workload, phases):
    """Over-budget task on the DRAM tier, progressive direct RPQ: the partitions land
    in byte phases, the fetch threads index each run as its phases arrive, and every key range that has
    fully arrived in all runs is merged in RPQ rounds while later phases still come in. Equal keys across
    the phase bounds (wordcount: few distinct words) must not be split or lost; phases=0 turns it off (the
    plain direct RPQ after the whole fetch)."""
    from uda_amd.utils.mof import write_mof
    p = UdaProvider()
    try:
        if workload == "secondary":
            maps = datagen.secondary_sort(num_maps=16, reducers=1, rows_per_map=6000, seed=9)
        else:
            maps = datagen.wordcount(num_maps=16, reducers=1, words_per_map=20000, seed=9)
        job = f"job_pd{workload}{phases}"
        ids = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_{job}_m_{i:06d}_0"
            path, _ = write_mof(str(tmp_path), mid, parts)
            p.add_mof_file(job, mid, path)
            ids.append(mid)
        conf = {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.merge.bytes": 400_000,
                "mapred.uda.gpu.spill": "host"}
        if phases:
            conf["mapred.uda.gpu.hybrid.progressive.phases"] = phases
        else:
            conf["mapred.uda.gpu.hybrid.progressive"] = 0
        recs, st, c = run_reduce("h", job, ids, 0, datagen.TEXT, conf=conf, kv_buf_size=8192)
        assert st["hybrid_direct"] == 1 and st["lpqs"] == 0 and st["rpq_rounds"] >= 2, st
        assert st["merge_path"] == ("staged-progressive-direct" if phases else "staged"), st
        want = sorted((kv for m in maps for kv in m[0]), key=datagen.sort_key(datagen.TEXT))
        kf = datagen.sort_key(datagen.TEXT)
        assert [kf(kv) for kv in recs] == [kf(kv) for kv in want]
        assert sorted(recs) == sorted(want)
        assert st["maps_fetched"] == 16
    finally:
        p.close()


def test_consumer_gpu_hybrid_checkpoint_resume(require_gpu, tmp_path, monkeypatch):
    """mapred.uda.lpq.checkpoint with the GPU hybrid merge (disk tier): attempt 0 fails after its
    2nd LPQ spill; attempt 1 restores both spills (data + sparse index), fetches only the other MOFs
    and delivers the same merged output; nothing is left behind after success."""
    from uda_amd.bridge import UdaConsumer, UdaFallback
    from uda_amd.utils.mof import write_mof
    p = UdaProvider()
    try:
        maps = datagen.secondary_sort(num_maps=12, reducers=2, rows_per_map=2000, seed=6)
        ids = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_hck_m_{i:06d}_0"
            path, _ = write_mof(str(tmp_path), mid, parts)
            p.add_mof_file("job_hck", mid, path)
            ids.append(mid)
        d1 = tmp_path / "ld1"
        d1.mkdir()
        conf = {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.merge.bytes": 300_000,
                "mapred.uda.gpu.spill": "disk", "mapred.uda.lpq.checkpoint": 1}
        kw = dict(conf=conf, kv_buf_size=8192, local_dirs=(str(d1),))
        monkeypatch.setenv("UDA_FAULT_LPQ_DONE", "2")
        c = UdaConsumer(len(ids), "job_hck", "attempt_job_hck_r_000000_0", datagen.TEXT, **kw)
        for m in ids:
            c.fetch("h", "job_hck", m, 0)
        with pytest.raises(UdaFallback, match="injected"):
            c.wait(60)
        c.close()
        monkeypatch.delenv("UDA_FAULT_LPQ_DONE")
        lines = (d1 / "uda.attempt_job_hck_r_000000.lpq.manifest").read_text().splitlines()
        assert [ln.split()[:2] for ln in lines] == [["glpq", "0"], ["glpq", "1"]]
        restored = {m for ln in lines for m in ln.split()[4].split(",")}
        recs, st, _ = run_reduce("h", "job_hck", ids, 0, datagen.TEXT, **kw)
        assert st["restored_lpqs"] == 2 and st["restored_maps"] == len(restored) > 0, st
        assert st["maps_fetched"] == len(ids)
        want = sorted((kv for m in maps for kv in m[0]), key=datagen.sort_key(datagen.TEXT))
        kf = datagen.sort_key(datagen.TEXT)
        assert [kf(kv) for kv in recs] == [kf(kv) for kv in want]
        assert sorted(recs) == sorted(want)
        assert not os.listdir(d1)
    finally:
        p.close()


def test_checkpoint_resume_with_device_resident_mofs(require_gpu, tmp_path, monkeypatch):
    """A resumed attempt (LPQ checkpoint of an earlier staged attempt) whose MOFs are now HBM-resident
    must not take the device-fetch path (it would wait forever for the FETCHes the checkpoint drops,
    or leave the restored records out): it merges the restored runs on the staged path."""
    from uda_amd.bridge import UdaConsumer, UdaFallback
    from uda_amd.utils.mof import read_index, write_mof
    p = UdaProvider()
    try:
        maps = datagen.secondary_sort(num_maps=10, reducers=1, rows_per_map=2000, seed=9)
        ids, files = [], []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_hdv_m_{i:06d}_0"
            path, _ = write_mof(str(tmp_path), mid, parts)
            p.add_mof_file("job_hdv", mid, path)
            ids.append(mid)
            files.append(path)
        d1 = tmp_path / "ld1"
        d1.mkdir()
        conf = {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.merge.bytes": 300_000,
                "mapred.uda.gpu.spill": "disk", "mapred.uda.lpq.checkpoint": 1}
        kw = dict(conf=conf, kv_buf_size=8192, local_dirs=(str(d1),))
        monkeypatch.setenv("UDA_FAULT_LPQ_DONE", "2")
        c = UdaConsumer(len(ids), "job_hdv", "attempt_job_hdv_r_000000_0", datagen.TEXT, **kw)
        for m in ids:
            c.fetch("h", "job_hdv", m, 0)
        with pytest.raises(UdaFallback, match="injected"):
            c.wait(60)
        c.close()
        monkeypatch.delenv("UDA_FAULT_LPQ_DONE")
        for mid, path in zip(ids, files):  # the same map outputs, now in HBM (descriptor-servable)
            with open(path, "rb") as f:
                p.add_mof_device("job_hdv", mid, f.read(), read_index(path + ".index"))
        recs, st, _ = run_reduce("h", "job_hdv", ids, 0, datagen.TEXT, timeout=90, **kw)
        assert st["restored_lpqs"] == 2 and st["device_descriptors"] == 0, st
        want = sorted((kv for m in maps for kv in m[0]), key=datagen.sort_key(datagen.TEXT))
        kf = datagen.sort_key(datagen.TEXT)
        assert [kf(kv) for kv in recs] == [kf(kv) for kv in want]
        assert sorted(recs) == sorted(want)
    finally:
        p.close()


def test_consumer_gpu_device_alloc_fault_fails_once(require_gpu, tmp_path, monkeypatch):
    from uda_amd.bridge import UdaConsumer, UdaFallback
    from uda_amd.utils.mof import write_mof
    p = UdaProvider()
    try:
        maps = datagen.wordcount(num_maps=3, reducers=1, words_per_map=1000, seed=2)
        ids = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_fa_m_{i:06d}_0"
            path, _ = write_mof(str(tmp_path), mid, parts)
            p.add_mof_file("job_fa", mid, path)
            ids.append(mid)
        monkeypatch.setenv("UDA_FAULT_DEVICE_ALLOC", "1")
        c = UdaConsumer(len(ids), "job_fa", "attempt_job_fa_r_000000_0", datagen.TEXT,
                        conf={"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.prewarm": 0})
        for m in ids:
            c.fetch("h", "job_fa", m, 0)
        with pytest.raises(UdaFallback, match="injected"):
            c.wait(60)
        c.close()
        assert c.failure_calls == 1
    finally:
        p.close()


@pytest.mark.parametrize("maps", [2, 5, 64, 128])
def test_generic_kway_matches_pairwise_tree(require_gpu, monkeypatch, maps):
    """The single-pass K-way merge of generic keys (sampled cells, LDS-staged key bytes after the
    cell's common prefix) orders records exactly like the pairwise merge tree (UDA_GKWAY=0) and the
    CPU heap merge, for long common prefixes, duplicate-heavy keys and fixed-width keys."""
    sec = [s[0] for s in datagen.streams(datagen.secondary_sort(maps, 1, 400, seed=maps))]
    wc = [s[0] for s in datagen.streams(datagen.wordcount(maps, 1, 300, seed=maps))]
    for runs in (sec, wc):
        g, _ = ops.merge_runs(runs, datagen.TEXT, "gpu")
        assert ops.last_stats["passes"] == 1
        monkeypatch.setenv("UDA_GKWAY", "0")
        t, _ = ops.merge_runs(runs, datagen.TEXT, "gpu")
        assert ops.last_stats["passes"] > 1 or maps <= 2
        monkeypatch.delenv("UDA_GKWAY")
        c, _ = ops.merge_runs(runs, datagen.TEXT, "cpu")
        assert g == t == c


@pytest.mark.parametrize("recurse", ["64", "8"])
def test_generic_kway_recursive_sample_merge(require_gpu, monkeypatch, recurse):
    """Large samples are merged by a nested K-way level (two levels with the lower threshold); the
    result must still equal the CPU heap merge."""
    monkeypatch.setenv("UDA_GKWAY_RECURSE", recurse)
    runs = [s[0] for s in datagen.streams(datagen.secondary_sort(24, 1, 1500, seed=31))]
    g, _ = ops.merge_runs(runs, datagen.TEXT, "gpu")
    assert ops.last_stats["passes"] == 1
    c, _ = ops.merge_runs(runs, datagen.TEXT, "cpu")
    assert g == c


@pytest.mark.parametrize("conf_extra", [
    {"mapred.uda.gpu.prewarm": 1, "mapred.uda.gpu.prewarm.pinned.mb": 64},
    {"mapred.uda.gpu.prewarm": 0, "mapred.uda.gpu.progressive.phases": 0},
    {"mapred.uda.gpu.merge.bytes": 200_000, "mapred.uda.gpu.spill": "host"},
])
def test_consumer_gpu_gate_and_prewarm(require_gpu, conf_extra):
    """The INIT-time prewarm and the phase / hybrid choices change when work happens, never what is
    delivered: the stream equals the CPU merge's, including a direct-RPQ hybrid task."""
    from uda_amd.utils.mof import encode_partitions
    p = UdaProvider()
    try:
        mp = datagen.secondary_sort(num_maps=10, reducers=2, rows_per_map=1500, seed=21)
        ids = []
        for i, parts in enumerate(datagen.streams(mp)):
            mid = f"attempt_g_m_{i:06d}_0"
            data, index = encode_partitions(parts)
            p.add_mof_memory("job_g2", mid, data, index)
            ids.append(mid)
        conf = {"mapred.uda.merge.backend": "gpu", **conf_extra}
        recs_gpu, st, _ = run_reduce("h", "job_g2", ids, 0, datagen.TEXT, conf=conf, max_buf_kb=16, min_buf_kb=16,
                                     kv_buf_size=8192)
        recs_cpu, _, _ = run_reduce("h", "job_g2", ids, 0, datagen.TEXT, max_buf_kb=16, min_buf_kb=16,
                                    kv_buf_size=8192)
        assert st["backend"] == "gpu" and st["maps_fetched"] == len(ids)
        assert [k for k, _ in recs_gpu] == [k for k, _ in recs_cpu]
        assert sorted(recs_gpu) == sorted(recs_cpu)
        if conf_extra.get("mapred.uda.gpu.prewarm") == 1:
            assert st["gpu_prewarm_ms"] >= 0, st
        if "mapred.uda.gpu.merge.bytes" in conf_extra:
            assert st["hybrid_direct"] == 1 and st["rpq_rounds"] >= 2, st
    finally:
        p.close()
