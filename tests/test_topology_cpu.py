"""CPU tier: host-thread placement on a multi-GPU node, and the per-rank record of a multi-GPU bench.

A fake 8 x MI355X node (two sockets, 64 cores / 128 CPUs each, SMT siblings numbered c and c + 128, four
GPUs per NUMA node) is described under UDA_SYSFS_ROOT. Every GPU must get a consumer CPU slice inside its
own NUMA node (where its delivery ring's pages are bound, sdma.h), the eight slices must be disjoint, and
whole cores (both SMT siblings) must go to one GPU.
"""
import os
import types

import pytest

import bench


def _fake_node(root, gpus_per_node=4, nodes=2, cores_per_node=64):
    cpus_total = nodes * cores_per_node
    for n in range(nodes):
        d = root / "sys/devices/system/node" / f"node{n}"
        d.mkdir(parents=True)
        lo = n * cores_per_node
        (d / "cpulist").write_text(f"{lo}-{lo + cores_per_node - 1},{cpus_total + lo}-{cpus_total + lo + cores_per_node - 1}\n")
    for c in range(cpus_total):
        for x in (c, c + cpus_total):
            t = root / "sys/devices/system/cpu" / f"cpu{x}" / "topology"
            t.mkdir(parents=True)
            (t / "thread_siblings_list").write_text(f"{c},{c + cpus_total}\n")
    kfd = root / "sys/class/kfd/kfd/topology/nodes"
    k = 0
    for n in range(nodes):  # CPU agents first, as KFD lists them
        (kfd / str(k)).mkdir(parents=True)
        (kfd / str(k) / "properties").write_text("cpu_cores_count 64\nsimd_count 0\nlocation_id 0\ndomain 0\n")
        k += 1
    buses = []
    for n in range(nodes):
        for g in range(gpus_per_node):
            bus = 0x05 + 0x10 * g + 0x80 * n
            buses.append((bus, n))
            (kfd / str(k)).mkdir(parents=True)
            (kfd / str(k) / "properties").write_text(f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {bus << 8}\n"
                                                      f"domain 0\ndrm_render_minor {128 + len(buses) - 1}\n")
            p = root / "sys/bus/pci/devices" / f"0000:{bus:02x}:00.0"
            p.mkdir(parents=True)
            (p / "numa_node").write_text(f"{n}\n")
            k += 1
    return buses, cpus_total


def test_eight_gpus_get_disjoint_numa_local_consumer_slices(native, tmp_path, monkeypatch):
    buses, total = _fake_node(tmp_path)
    monkeypatch.setenv("UDA_SYSFS_ROOT", str(tmp_path))
    plan = native.topology_plan([])
    assert [p["bdf"] for p in plan] == [f"0000:{b:02x}:00.0" for b, _ in sorted(buses)]
    seen = set()
    for p in plan:
        node = p["numa_node"]
        node_cpus = set(native.parse_cpulist((tmp_path / f"sys/devices/system/node/node{node}/cpulist").read_text()))
        cpus = set(p["cpus"])
        assert len(cpus) == 32, p            # 16 cores x 2 threads: a quarter of the socket
        assert cpus <= node_cpus, p          # NUMA-local: on the node its ring's pages live on
        assert not (cpus & seen), p          # disjoint from every other GPU's slice
        assert all(((c + total) % (2 * total) in cpus) for c in cpus), p  # whole cores
        seen |= cpus
    assert len({p["numa_node"] for p in plan}) == 2 and len(plan) == 8
    # an affinity mask (a container's cpuset) narrows the slices, which stay disjoint
    allowed = list(range(0, 32)) + list(range(128, 160)) + list(range(64, 96)) + list(range(192, 224))
    plan2 = native.topology_plan(sorted(allowed))
    got = [set(p["cpus"]) for p in plan2]
    assert all(got) and sum(len(g) for g in got) == len(allowed)
    assert all(not (a & b) for i, a in enumerate(got) for b in got[i + 1:])


def test_usable_gpus_are_the_openable_render_nodes(native, tmp_path, monkeypatch):
    """A one-GPU container on an 8-GPU host sees the whole KFD topology but opens one render node: the
    node daemons and the consumer slices count only that one (no HIP call in the front end)."""
    buses, _ = _fake_node(tmp_path)
    monkeypatch.setenv("UDA_SYSFS_ROOT", str(tmp_path))
    assert native.usable_gpu_bdfs() == []
    dri = tmp_path / "dev/dri"
    dri.mkdir(parents=True)
    (dri / "renderD131").write_bytes(b"")  # the 4th GPU (render minor 128 + 3)
    assert native.usable_gpu_bdfs() == [f"0000:{buses[3][0]:02x}:00.0"]
    for m in range(128, 136):
        (dri / f"renderD{m}").write_bytes(b"")
    assert len(native.usable_gpu_bdfs()) == 8


def test_cpulist_roundtrip(native):
    assert native.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert native.format_cpulist([0, 1, 2, 3, 8, 10, 11]) == "0-3,8,10-11"
    assert native.format_cpulist([]) == ""


def _record(ranks=8, rounds=4):
    det = []
    for r in range(ranks):
        det.append({"rank": r, "device": r, "numa_node": r // 4, "consumer_cpus": "0-15", "delivery": "sdma[...]",
                    "exchange": "ipc", "exchange_why": "--exchange ipc (default)", "peer_send_bytes": [1] * ranks,
                    "round_comm_ms": [1.0] * rounds, "round_merge_ms": [1.0] * rounds, "wall_ms": 1.0,
                    "comm_ms": 1.0, "merge_ms": 1.0, "d2h_ms": 1.0, "wait_out_ms": 0.0, "bytes_in": 10})
    return {"ranks": ranks, "config": {"rounds": rounds}, "peer_access": [[1] * ranks] * ranks, "ranks_detail": det}


def test_bench_record_schema():
    """The fields the first 8-GPU record must carry per rank."""
    assert bench.record_problems(_record()) == []
    bad = _record()
    del bad["ranks_detail"][3]["consumer_cpus"]
    bad["ranks_detail"][5]["peer_send_bytes"] = [1, 2]
    bad["ranks_detail"].pop()
    probs = bench.record_problems(bad)
    assert any("rank 3: consumer_cpus" in p for p in probs)
    assert any("rank 5: peer_send_bytes" in p for p in probs)
    assert any("7 entries for 8 ranks" in p for p in probs)


def test_rank_detail_from_a_job_without_gpu(native):
    """rank_detail() builds its record from the job's own accessors (no GPU here: no PCI address)."""
    stats = [{"round_comm_ms": [1.0, 2.0], "round_merge_ms": [3.0, 4.0], "wall_ms": 10.0, "comm_ms": 3.0,
              "merge_ms": 7.0, "d2h_ms": 1.0, "wait_out_ms": 0.5, "bytes_in": 100}] * 2
    job = types.SimpleNamespace(ipc_fallback=None, job=types.SimpleNamespace(
        delivery_name="sdma[numa=0 engines=2 h2d=3] ring=N0", exchange_name="ipc",
        peer_send_bytes=lambda: [0, 5]))
    ctx = types.SimpleNamespace(world=2, rank=1)
    args = types.SimpleNamespace(exchange="ipc")
    d = bench.rank_detail(args, ctx, job, 0, stats)
    assert d["round_comm_ms"] == [1.0, 2.0] and d["peer_send_bytes"] == [0, 5]
    assert d["exchange_why"].startswith("--exchange ipc") and d["numa_node"] == -1
    rec = {"ranks": 1, "config": {"rounds": 2}, "peer_access": [], "ranks_detail": [dict(d, rank=0, peer_send_bytes=[0])]}
    assert bench.record_problems(rec) == []
