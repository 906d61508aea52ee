"""Multi-process paths on the CPU: the torch.distributed control plane the bench uses between GPU
ranks (gloo, world 2), and the TCP transport with the MOFSupplier and the NetMerger in different
processes (the reference's cross-node shuffle, RDMAServer/RDMAClient, over sockets)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from uda_amd.bridge import UdaConsumer, UdaFallback
from uda_amd.utils import datagen
from uda_amd.utils.ifile import decode_stream  # noqa: F401
from uda_amd.utils.mof import write_mof

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _control_plane_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import numpy as np

    from uda_amd.parallel.dist import init_from_env
    from uda_amd.parallel.plan import round_bounds
    ctx = init_from_env()
    try:
        uid = ctx.broadcast_bytes(b"unique-id-from-rank0" if rank == 0 else None)
        g = ctx.all_gather_object({"rank": rank})
        sums = ctx.sum_u64([(1 << 63) + rank, 5])
        mx = ctx.max_float(float(rank) + 0.5)
        # the bench's bound planning: every rank contributes key samples per destination
        rng = np.random.default_rng(rank)
        local = [np.sort(rng.integers(0, 2**63, size=(50, 2), dtype=np.uint64), axis=0) for _ in range(world)]
        gathered = ctx.all_gather_object(local)
        per_dest = [np.concatenate([gg[d] for gg in gathered]) for d in range(world)]
        bounds = round_bounds(per_dest, 4)
        q.put((rank, uid, [x["rank"] for x in g], sums, mx, bounds.tobytes()))
        ctx.barrier()
    finally:
        ctx.close()


def test_control_plane_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_control_plane_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        _, uid, ranks, sums, mx, bounds = res[r]
        assert uid == b"unique-id-from-rank0"
        assert ranks == [0, 1]
        assert sums == [((1 << 63) * 2 + 1) % (1 << 64), 10]
        assert mx == 1.5
    assert res[0][5] == res[1][5]  # identical round bounds on every rank


PROVIDER = r"""
import json, sys
sys.path.insert(0, sys.argv[3])
from uda_amd.bridge import UdaProvider
p = UdaProvider(transport="tcp", data_port=int(sys.argv[1]))
for job, mid, path in json.loads(sys.argv[2]):
    p.add_mof_file(job, mid, path)
print("READY", flush=True)
sys.stdin.read()
p.close()
print(p.stats(), flush=True)
"""


@pytest.fixture
def tcp_provider(tmp_path):
    procs = []

    def start(mofs):
        port = _free_port()
        proc = subprocess.Popen([sys.executable, "-c", PROVIDER, str(port), json.dumps(mofs), ROOT],
                                stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
        assert proc.stdout.readline().strip() == "READY"
        procs.append(proc)
        return port, proc

    yield start
    for proc in procs:
        if proc.poll() is None:
            proc.stdin.close()
            try:
                proc.wait(timeout=30)
            except subprocess.TimeoutExpired:
                proc.kill()


@pytest.mark.parametrize("codec", [None, "lzo"])
def test_tcp_transport_across_processes(tmp_path, tcp_provider, codec):
    maps = datagen.secondary_sort(num_maps=7, reducers=3, rows_per_map=800, seed=17)
    job = "job_tcp_" + (codec or "raw")
    mofs = []
    for i, parts in enumerate(datagen.streams(maps)):
        mid = f"attempt_{job}_m_{i:06d}_0"
        path, _ = write_mof(str(tmp_path), mid, parts, codec=codec)
        mofs.append((job, mid, path))
    port, proc = tcp_provider(mofs)
    consumers = [UdaConsumer(len(mofs), job, f"attempt_{job}_r_{r:06d}_0", datagen.TEXT, codec=codec,
                             transport="tcp", data_port=port, max_buf_kb=16, kv_buf_size=16384)
                 for r in range(3)]
    for r, c in enumerate(consumers):  # all reducers fetch concurrently over one connection each
        for _, mid, _ in mofs:
            c.fetch("127.0.0.1", job, mid, r)
    kf = datagen.sort_key(datagen.TEXT)
    for r, c in enumerate(consumers):
        recs = c.wait(120)
        st = c.close()
        want = sorted((kv for m in maps for kv in m[r]), key=kf)
        assert [kf(kv) for kv in recs] == [kf(kv) for kv in want]
        assert sorted(recs) == sorted(want)
        assert st["maps_fetched"] == len(mofs)
    proc.stdin.close()
    assert proc.wait(timeout=30) == 0
    stats = json.loads(proc.stdout.read().strip().splitlines()[-1])
    assert stats["bytes_served"] > 0


def test_tcp_unreachable_provider_fails_once():
    port = _free_port()  # nothing listens here
    c = UdaConsumer(1, "job_tcp_none", "attempt_job_tcp_none_r_000000_0", datagen.TEXT, transport="tcp",
                    data_port=port)
    c.fetch("127.0.0.1", "job_tcp_none", "attempt_job_tcp_none_m_000000_0", 0)
    with pytest.raises(UdaFallback):
        c.wait(60)
    c.close()
    assert c.failure_calls == 1


def test_bench_self_launches_one_process_per_gpu():
    """`python bench.py --gpus N` without torchrun starts N rank processes itself."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--launch-selftest"],
                         capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stderr
    ranks = [json.loads(line) for line in out.stdout.splitlines() if line.startswith("{")]
    assert sorted(int(r["RANK"]) for r in ranks) == [0, 1, 2]
    assert {r["WORLD_SIZE"] for r in ranks} == {"3"}
    assert {r["MASTER_ADDR"] for r in ranks} == {"127.0.0.1"}
    assert len({r["MASTER_PORT"] for r in ranks}) == 1
    assert all(r["LOCAL_RANK"] == r["RANK"] for r in ranks)


def test_bench_refuses_world_mismatch():
    """A launcher that started a different number of ranks than --gpus asks for is an error."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                         capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 2
    assert "launcher started 1 rank" in out.stderr


def test_tcp_providers_share_a_port_on_distinct_addresses():
    """One provider per GPU on one node: each listens on the job's data port at its own loopback
    address (mapred.uda.provider.bind.address), as providers of different hosts do; a reduce task
    fetches each map from the provider that holds it."""
    import socket

    from uda_amd.bridge import UdaProvider
    from uda_amd.utils.mof import encode_partitions
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    maps = datagen.secondary_sort(num_maps=6, reducers=2, rows_per_map=500, seed=23)
    job = "job_bind_0001"
    provs = [UdaProvider(conf={"mapred.uda.provider.bind.address": f"127.0.0.{k + 1}"}, transport="tcp",
                         data_port=port) for k in range(2)]
    try:
        for i, parts in enumerate(datagen.streams(maps)):
            data, index = encode_partitions(parts)
            provs[i % 2].add_mof_memory(job, f"attempt_{job}_m_{i:06d}_0", data, index)
        c = UdaConsumer(len(maps), job, f"attempt_{job}_r_000001_0", datagen.TEXT, transport="tcp", data_port=port)
        for i in range(len(maps)):
            c.fetch(f"127.0.0.{i % 2 + 1}", job, f"attempt_{job}_m_{i:06d}_0", 1)
        recs = c.wait(60)
        c.close()
        kf = datagen.sort_key(datagen.TEXT)
        want = sorted((kv for m in maps for kv in m[1]), key=kf)
        assert [kf(kv) for kv in recs] == [kf(kv) for kv in want]
    finally:
        for p in provs:
            p.close()


def test_tcp_connections_and_by_reference_answers(native, tmp_path):
    """Several TCP connections per provider (mapred.uda.tcp.connections) and answers sent by reference
    (sendfile of the MOF file, the registered memory itself) deliver the same bytes as one connection
    with chunk copies; every byte lands at its offset (out-of-order completions across connections)."""
    import random
    import socket
    import zlib
    from uda_amd.bridge import UdaProvider
    from uda_amd.utils.mof import write_index
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    rnd = random.Random(7)
    sizes = [rnd.randrange(1, 3 << 20) for _ in range(6)]
    blobs = [rnd.randbytes(n) for n in sizes]
    for copy in ("0", "1"):
        p = UdaProvider(transport="tcp", data_port=port,
                        conf={"mapred.uda.provider.bind.address": "127.0.0.1", "mapred.uda.daemon": "0",
                              "mapred.uda.provider.copy.serve": copy})
        try:
            ids = []
            for i, b in enumerate(blobs):
                if i % 2:
                    p.add_mof_memory("job_tcp", f"m{i}", b, [(0, len(b), len(b))])
                else:
                    d = tmp_path / f"m{i}"
                    d.mkdir(exist_ok=True)
                    (d / "file.out").write_bytes(b)
                    write_index(str(d / "file.out.index"), [(0, len(b), len(b))])
                    p.add_mof_file("job_tcp", f"m{i}", str(d / "file.out"))
                ids.append(f"m{i}")
            want = sum(b[k] for b in [b"".join(blobs)] for k in range(0, len(b), 4096))
            for conns, chunk, depth, par in ((1, 1 << 20, 1, 1), (4, 256 << 10, 4, 3), (3, 1 << 20, 8, 6)):
                tot, sec, got = native.tcp_fetch_probe("127.0.0.1", port, "job_tcp", ids, 0, sizes, chunk, depth,
                                                       conns, par)
                assert tot == sum(sizes) and got == want, (copy, conns, chunk)
        finally:
            p.close()


def test_tcp_dead_host_does_not_delay_live_hosts(native, tmp_path):
    """the TCP client opened a host's connections (5 tries each, ~1.5 s) while holding
    its client-wide lock, so one unreachable provider stalled every other host's fetches for ~6 s. Now a
    host's connections open outside the lock: a live host's fetch issued while the dead host is still
    being tried completes at once, and the dead host, once failed, fails the next fetch at once (backoff)."""
    import random
    import socket
    from uda_amd.bridge import UdaProvider
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    blob = random.Random(3).randbytes(1 << 20)
    p = UdaProvider(transport="tcp", data_port=port,
                    conf={"mapred.uda.provider.bind.address": "127.0.0.1", "mapred.uda.daemon": "0"})
    try:
        p.add_mof_memory("job_dead", "m0", blob, [(0, len(blob), len(blob))])
        # nothing listens on 127.0.0.3:<port> (the provider is bound to 127.0.0.1 only): refused at once
        live_ms, dead_err, dead_ms, dead2_ms = native.tcp_dead_host_probe(
            "127.0.0.1", f"127.0.0.3:{port}", port, "job_dead", "m0", 0, len(blob))
        assert dead_err, "the dead host's fetch must fail"
        assert dead_ms > 1000, dead_ms  # it was really tried (5 tries with backoff)
        assert live_ms < 500, live_ms   # not held behind those tries
        assert dead2_ms < 200, dead2_ms  # backoff: fails at once
    finally:
        p.close()


def test_declined_descriptor_ack_keeps_partition_lengths(native):
    """A provider declining a descriptor fetch (kNotDeviceResident, -12: its HBM store is full) answers
    with the partition's lengths, so the reducer knows how many bytes to fetch instead. Over TCP the
    error ack used to carry only the status and text: 23 of 32 partitions were then "fetched" as 0
    bytes and the merged output silently lacked them (r6 node run with a store smaller than the MOFs)."""
    got = native.ack_roundtrip(-12, 1000, 993, 0, 4096, "/d:1/m_3/file.out", "provider HBM store: full: 3 of 3 GB")
    assert got["status"] == -12 and got["part_len"] == 993 and got["raw_len"] == 1000 and got["mof_offset"] == 4096
    assert got["path"] == "/d:1/m_3/file.out"  # where the bytes are (a reducer on the node may read them)
    assert got["error"] == "provider HBM store: full: 3 of 3 GB"  # path and text may contain ':'
    ok = native.ack_roundtrip(0, 10, 8, 8, 0, "/a:b/file.out", "")
    assert (ok["status"], ok["part_len"], ok["sent"], ok["path"]) == (0, 8, 8, "/a:b/file.out")
    err = native.ack_roundtrip(-2, 0, 0, 0, 0, "", "cannot resolve MOF j/m/0")
    assert err["status"] == -2 and err["error"] == "cannot resolve MOF j/m/0"


def test_declined_partitions_are_read_locally_only_from_own_regular_files(native, tmp_path):
    """mapred.uda.gpu.fetch.local.read: a reducer reads a declined partition from the MOF file the provider
    named only when the provider is on this node and the file is a regular file of its own user that holds
    the partition -- never through a symlink, never past the file's end, never a relative path."""
    import socket
    assert native.mof_host_is_local("127.0.0.1:9011") and native.mof_host_is_local("localhost")
    assert native.mof_host_is_local(socket.gethostname())
    assert not native.mof_host_is_local("10.255.255.1:9011")
    mof = tmp_path / "file.out"
    mof.write_bytes(b"x" * 4096)
    assert native.local_mof_readable(str(mof), 0, 4096)
    assert native.local_mof_readable(str(mof), 1000, 3096)
    assert not native.local_mof_readable(str(mof), 1000, 3097)  # past the end
    link = tmp_path / "link.out"
    link.symlink_to(mof)
    assert not native.local_mof_readable(str(link), 0, 10)  # a symlink planted in the path
    assert not native.local_mof_readable("file.out", 0, 10)  # relative
    assert not native.local_mof_readable(str(tmp_path), 0, 0)  # a directory
    if os.geteuid() == 0:  # a file of another user
        other = tmp_path / "other.out"
        other.write_bytes(b"y" * 4096)
        os.chown(other, 65534, 65534)
        assert not native.local_mof_readable(str(other), 0, 10)
