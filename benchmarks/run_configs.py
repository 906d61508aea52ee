#!/usr/bin/env python3
"""Benchmarks for the BASELINE.json configs other than the flagship (bench.py).

  wordcount_loopback  uda_standalone wordcount on CPU loopback: provider + R NetMergers in one
                      process through the UdaBridge C ABI (the JNI plumbing path), heap merge.
  wordcount_tcp       the same with the MOFSupplier in another process, over the TCP transport.
  cpu_reference       in-house baseline: the reference algorithm (single-threaded heap k-way merge,
                      write_kv_to_stream packing) on TeraSort runs on this host's CPU.
  secondary_sort      variable-length Text keys with long common prefixes + partition skew: GPU generic
                      merge (F1/F2/F3/F4 kernels) vs the CPU heap merge on the same runs.
  decode              F6 Snappy / LZO1X block decode on the device vs the host decoder.
  netmerger           secondary-sort data through provider -> NetMerger -> dataFromUda: CPU heap merge vs
                      GPU backend (online and hybrid LPQ/RPQ).
  aio                 AsyncIO (io_uring / thread pool, O_DIRECT) read bandwidth vs sequential pread.
  spill               TeraSort whose map outputs live in pinned host DRAM (the spill tier used when a
                      job exceeds HBM): rounds are streamed H2D, merged on the GPU, delivered D2H.

Each prints one JSON line per result. Data is synthetic (native generators, csrc/engine/datagen.cc).
"""
from __future__ import annotations

import argparse
import json
import sys
import threading
import resource
import time
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def wordcount_loopback(args) -> dict:
    from uda_amd import native
    from uda_amd.bridge import UdaConsumer, UdaProvider
    from uda_amd.utils.datagen import TEXT
    from uda_amd.utils.mof import encode_partitions

    n = native()
    maps, reducers = args.maps, args.reducers
    rows = int(args.gb * 1e9 / maps / 17)  # ~17 B per (word, 1) IFile record
    t0 = time.perf_counter()
    runs = n.generate_runs("wordcount", maps, reducers, rows, 7)
    gen_s = time.perf_counter() - t0
    prov = UdaProvider()
    total = 0
    for m, parts in enumerate(runs):
        data, index = encode_partitions(parts)
        total += len(data) - 2 * len(parts)
        prov.add_mof_memory("job_wc", f"attempt_wc_m_{m:06d}_0", data, index)
    consumers = [UdaConsumer(maps, "job_wc", f"attempt_wc_r_{r:06d}_0", TEXT, keep_records=False)
                 for r in range(reducers)]
    t0 = time.perf_counter()
    for r, c in enumerate(consumers):
        for m in range(maps):
            c.fetch("localhost", "job_wc", f"attempt_wc_m_{m:06d}_0", r)
    for c in consumers:
        c.wait(3600)
    wall = time.perf_counter() - t0
    stats = [c.close() for c in consumers]
    prov.close()
    delivered = sum(s["bytes_delivered"] for s in stats) - 2 * reducers
    assert delivered == total, (delivered, total)
    return {"config": "uda_standalone wordcount CPU loopback", "gb": round(total / 1e9, 3),
            "maps": maps, "reducers": reducers, "wall_s": round(wall, 3),
            "shuffle_merge_gbps": round(total / wall / 1e9, 3), "gen_s": round(gen_s, 1),
            "records": sum(s["records"] for s in stats), "backend": "cpu heap merge, loopback transport"}


TCP_PROVIDER = r"""
import json, sys
sys.path.insert(0, sys.argv[3])
from uda_amd.bridge import UdaProvider
p = UdaProvider(transport="tcp", data_port=int(sys.argv[1]))
for job, mid, path in json.loads(sys.argv[2]):
    p.add_mof_file(job, mid, path)
print("READY", flush=True)
sys.stdin.read()
p.close()
"""


def wordcount_tcp(args) -> dict:
    """wordcount with the MOFSupplier in another process: the socket transport (the reference's
    cross-node RDMA path, here TCP over the host's loopback interface)."""
    import socket
    import subprocess
    import tempfile

    from uda_amd import native
    from uda_amd.bridge import UdaConsumer
    from uda_amd.utils.datagen import TEXT
    from uda_amd.utils.mof import write_mof
    n = native()
    maps, reducers = args.maps, args.reducers
    rows = int(args.gb * 1e9 / maps / 17)
    runs = n.generate_runs("wordcount", maps, reducers, rows, 7)
    tmp = tempfile.mkdtemp(prefix="uda_tcp_", dir=args.dir)
    mofs, total = [], 0
    for m, parts in enumerate(runs):
        mid = f"attempt_tcp_m_{m:06d}_0"
        path, _ = write_mof(tmp, mid, parts)
        mofs.append(("job_tcp", mid, path))
        total += sum(len(p) - 2 for p in parts)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prov = subprocess.Popen([sys.executable, "-c", TCP_PROVIDER, str(port), json.dumps(mofs), root],
                            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        assert prov.stdout.readline().strip() == "READY"
        consumers = [UdaConsumer(maps, "job_tcp", f"attempt_tcp_r_{r:06d}_0", TEXT, keep_records=False,
                                 transport="tcp", data_port=port) for r in range(reducers)]
        t0 = time.perf_counter()
        for r, c in enumerate(consumers):
            for _, mid, _ in mofs:
                c.fetch("127.0.0.1", "job_tcp", mid, r)
        for c in consumers:
            c.wait(3600)
        wall = time.perf_counter() - t0
        stats = [c.close() for c in consumers]
    finally:
        prov.stdin.close()
        prov.wait(timeout=60)
    delivered = sum(st["bytes_delivered"] for st in stats) - 2 * reducers
    assert delivered == total, (delivered, total)
    return {"config": "wordcount, MOFSupplier in a separate process, TCP transport", "gb": round(total / 1e9, 3),
            "maps": maps, "reducers": reducers, "wall_s": round(wall, 3),
            "shuffle_merge_gbps": round(total / wall / 1e9, 3)}


def cpu_reference(args) -> dict:
    from uda_amd import native
    n = native()
    rows = int(args.gb * 1e9 / 104 / args.maps)
    runs = [p[0] for p in n.generate_runs("terasort", args.maps, 1, rows, 3)]
    nbytes = sum(len(r) - 2 for r in runs)
    t0 = time.perf_counter()
    out, lens = n.cpu_merge(runs, "org.apache.hadoop.io.Text", 1 << 20)
    dt = time.perf_counter() - t0
    assert len(out) == nbytes + 2
    return {"config": "reference algorithm: 1-thread heap k-way merge (CPU)", "gb": round(nbytes / 1e9, 3),
            "runs": args.maps, "merge_s": round(dt, 3), "merge_gbps": round(nbytes / dt / 1e9, 3),
            "buffers": len(lens)}


def secondary_sort(args) -> dict:
    from uda_amd import native, ops
    n = native()
    rows = int(args.gb * 1e9 / 100 / args.maps)
    gen = n.generate_runs("secondary", args.maps, 2, rows, 5)
    runs = [m[0] for m in gen]  # reducer 0 receives the skewed majority
    nbytes = sum(len(r) - 2 for r in runs)
    # first full-size call: allocates the merger's HBM workspace (cached per process afterwards, as
    # the NetMerger's pooled workspace is across reduce tasks)
    ops.merge_runs(runs, "org.apache.hadoop.io.Text", "gpu")
    cold_ms = ops.last_stats["merge_ms"]
    res = {}
    for dev in ("gpu", "cpu"):
        t0 = time.perf_counter()
        body, cuts = ops.merge_runs(runs, "org.apache.hadoop.io.Text", dev)
        dt = time.perf_counter() - t0
        res[dev] = (dt, body)
        if dev == "gpu":
            dev_ms = ops.last_stats["merge_ms"]
    assert res["gpu"][1] == res["cpu"][1], "GPU and CPU merges differ"
    return {"config": "secondary sort: variable-length Text keys, long common prefixes, 60% skew to reducer 0",
            "gb": round(nbytes / 1e9, 3), "runs": args.maps,
            "gpu_s_incl_h2d_d2h": round(res["gpu"][0], 3), "cpu_heap_s": round(res["cpu"][0], 3),
            "gpu_gbps": round(nbytes / res["gpu"][0] / 1e9, 3), "cpu_gbps": round(nbytes / res["cpu"][0] / 1e9, 3),
            "gpu_device_merge_ms": round(dev_ms, 1), "gpu_device_merge_gbps": round(nbytes / dev_ms / 1e6, 2),
            "gpu_device_merge_first_call_ms": round(cold_ms, 1),
            "byte_identical": True}


def decode(args) -> dict:
    """F6: device block decode of block-compressed IFile runs (secondary-sort data) vs host decode."""
    from uda_amd import native
    n = native()
    codec = {"snappy": 1, "lzo": 2}[args.codec]
    rows = int(args.gb * 1e9 / 100 / args.maps)
    runs = [m[0] for m in n.generate_runs("secondary", args.maps, 1, rows, 5)]
    t0 = time.perf_counter()
    streams = [n.block_compress(codec, r, 256 * 1024) for r in runs]
    comp_s = time.perf_counter() - t0
    raw = sum(len(r) for r in runs)
    comp = sum(len(s) for s in streams)
    n.gpu_block_decode(args.codec, streams[:1])  # warm up
    outs, blocks, ms = n.gpu_block_decode(args.codec, streams)
    assert outs == runs
    t0 = time.perf_counter()
    host = n.block_decompress(codec, streams[0], 1 << 20)
    host_s = (time.perf_counter() - t0) * len(streams)
    assert host == runs[0]
    return {"config": f"F6 device {args.codec} block decode, 256 KiB blocks, secondary-sort IFile data",
            "raw_gb": round(raw / 1e9, 3), "ratio": round(raw / comp, 2), "blocks": blocks,
            "device_decode_ms": round(ms, 1), "device_gbps_raw": round(raw / ms / 1e6, 1),
            "host_1thread_gbps_raw": round(raw / host_s / 1e9, 3), "host_compress_s": round(comp_s, 1)}


def netmerger(args) -> dict:
    """Secondary-sort data through the whole plugin path (provider -> loopback fetch -> NetMerger ->
    dataFromUda): CPU heap merge vs the GPU backend (online, and hybrid LPQ/RPQ with a small device
    budget)."""
    from uda_amd import native
    from uda_amd.bridge import UdaConsumer, UdaProvider
    from uda_amd.utils.datagen import TEXT
    from uda_amd.utils.mof import encode_partitions
    n = native()
    rows = int(args.gb * 1e9 / 100 / args.maps)
    runs = n.generate_runs("secondary", args.maps, 1, rows, 9)
    prov = UdaProvider()
    total = 0
    for m, parts in enumerate(runs):
        data, index = encode_partitions(parts)
        total += len(data) - 2
        prov.add_mof_memory("job_nm", f"attempt_nm_m_{m:06d}_0", data, index)
    out = {"config": "secondary sort through the NetMerger (loopback transport, 1 reducer)",
           "gb": round(total / 1e9, 3), "maps": args.maps}
    variants = [("cpu", {}), ("gpu_cold", {"mapred.uda.merge.backend": "gpu"}),
                ("gpu_second", {"mapred.uda.merge.backend": "gpu"}),
                ("gpu", {"mapred.uda.merge.backend": "gpu"}),
                ("gpu_drains_all", {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.fetch.drains": 0}),
                ("gpu_drains8_step8m", {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.fetch.drains": 8,
                                        "mapred.uda.gpu.early.h2d.step": 8 << 20}),
                ("gpu_hybrid_first", {"mapred.uda.merge.backend": "gpu",
                                      "mapred.uda.gpu.merge.bytes": max(1 << 20, total // 6),
                                      "mapred.uda.gpu.spill": "host"}),
                ("gpu_hybrid", {"mapred.uda.merge.backend": "gpu",
                                "mapred.uda.gpu.merge.bytes": max(1 << 20, total // 6),
                                "mapred.uda.gpu.spill": "host"}),
                ("gpu_hybrid_lpq", {"mapred.uda.merge.backend": "gpu",
                                    "mapred.uda.gpu.merge.bytes": max(1 << 20, total // 6),
                                    "mapred.uda.gpu.spill": "host", "mapred.uda.gpu.hybrid.direct": 0})]
    for i, (name, conf) in enumerate(variants):
        c = UdaConsumer(args.maps, "job_nm", f"attempt_nm_r_{i:06d}_0", TEXT, conf=conf, keep_records=False)
        r0 = resource.getrusage(resource.RUSAGE_SELF)
        t0 = time.perf_counter()
        for m in range(args.maps):
            c.fetch("localhost", "job_nm", f"attempt_nm_m_{m:06d}_0", 0)
        c.wait(3600)
        wall = time.perf_counter() - t0
        r1 = resource.getrusage(resource.RUSAGE_SELF)
        # CPU seconds the task burned (all threads): the GPU box runs under a 16-CPU CFS quota, and a
        # process that exceeds it inside a 100 ms period is stalled until the next one
        out[name + "_cpu_s"] = round(r1.ru_utime + r1.ru_stime - r0.ru_utime - r0.ru_stime, 3)
        st = c.close()
        print(f"# {name}: {wall * 1e3:.1f} ms, delivered {st['bytes_delivered'] - 2} of {total} "
              f"path={st.get('merge_path')}", file=sys.stderr, flush=True)
        assert st["bytes_delivered"] - 2 == total, (name, st)
        out[name + "_gbps"] = round(total / wall / 1e9, 3)
        out[name + "_merge_ms"] = round(st["merge_ms"], 1)
        out[name + "_fetch_ms"] = round(st["fetch_ms"], 1)
        if name.startswith("gpu"):
            out[name + "_phases_ms"] = {k: round(st["gpu_" + k + "_ms"], 1) for k in ("h2d", "device", "d2h_wait", "sink")}
        if name.startswith("gpu_hybrid"):
            out[name + "_direct"] = st.get("hybrid_direct")
        if name == "gpu_hybrid":
            out["hybrid_lpqs"] = st["lpqs"]
            out["hybrid_rpq_rounds"] = st["rpq_rounds"]
    prov.close()
    out.update(_netmerger_device_mofs(args, runs))
    if args.reducers > 1:
        out.update(_netmerger_concurrent(args, rows))
    return out


def _netmerger_device_mofs(args, runs) -> dict:
    """The same data with HBM-resident MOFs (the provider registers device memory): the reducer fetches
    partition descriptors and merges the partitions where they live, so only the merged output
    crosses PCIe (device fetch, generic-key merge with key-range rounds streamed out)."""
    from uda_amd.bridge import UdaConsumer, UdaProvider
    from uda_amd.utils.datagen import TEXT
    from uda_amd.utils.mof import encode_partitions
    prov = UdaProvider()
    total = 0
    for m, parts in enumerate(runs):
        data, index = encode_partitions(parts)
        total += len(data) - 2
        prov.add_mof_device("job_nmd", f"attempt_nmd_m_{m:06d}_0", data, index)
    out = {}
    conf = {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.fetch": "device"}
    for attempt in ("cold", "warm", "warm2"):
        c = UdaConsumer(args.maps, "job_nmd", f"attempt_nmd_r_000000_{attempt}", TEXT, conf=conf, keep_records=False)
        t0 = time.perf_counter()
        for m in range(args.maps):
            c.fetch("localhost", "job_nmd", f"attempt_nmd_m_{m:06d}_0", 0)
        c.wait(3600)
        wall = time.perf_counter() - t0
        st = c.close()
        assert st["bytes_delivered"] - 2 == total, (st["bytes_delivered"], total)
        out[f"gpu_hbm_mofs_{attempt}_gbps"] = round(total / wall / 1e9, 3)
        if attempt != "cold":
            out[f"gpu_hbm_mofs_{attempt}_stats"] = {k: st[k] for k in ("merge_path", "device_descriptors",
                                                                       "host_fetched_bytes", "gpu_device_ms",
                                                                       "gpu_d2h_wait_ms", "merge_ms", "fetch_ms")
                                                   if k in st}
    prov.close()
    return out


def _netmerger_concurrent(args, rows: int) -> dict:
    """The node view of the same path: `reducers` reduce tasks of one job run at once on one GPU (a
    TaskTracker's reduce slots), each its own NetMerger over its partition of every MOF. One task's
    input H2D overlaps another's output D2H, so the node uses both PCIe directions."""
    from uda_amd import native
    from uda_amd.bridge import UdaConsumer, UdaProvider
    from uda_amd.utils.datagen import TEXT
    from uda_amd.utils.mof import encode_partitions
    n, R = native(), args.reducers
    runs = n.generate_runs("secondary", args.maps, R, rows, 11)
    prov = UdaProvider()
    for m, parts in enumerate(runs):
        data, index = encode_partitions(parts)
        prov.add_mof_memory("job_nmc", f"attempt_nmc_m_{m:06d}_0", data, index)
    del runs
    out = {}
    for attempt in ("cold", "warm"):
        cons = [UdaConsumer(args.maps, "job_nmc", f"attempt_nmc_r_{r:06d}_{attempt}", TEXT,
                            conf={"mapred.uda.merge.backend": "gpu"}, keep_records=False) for r in range(R)]
        t0 = time.perf_counter()
        for m in range(args.maps):
            for r, c in enumerate(cons):
                c.fetch("localhost", "job_nmc", f"attempt_nmc_m_{m:06d}_0", r)
        for c in cons:
            c.wait(3600)
        wall = time.perf_counter() - t0
        stats = [c.close() for c in cons]
        total = sum(st["bytes_delivered"] - 2 for st in stats)
        out[f"gpu_{R}tasks_{attempt}_gbps"] = round(total / wall / 1e9, 3)
    out[f"gpu_{R}tasks_gb"] = round(total / 1e9, 3)
    prov.close()
    return out


def hybrid_budget(args) -> dict:
    """BASELINE config #4's mechanism on one GPU: one reduce task whose partition is several times its
    device budget. The map outputs are in host memory (the DRAM tier), mapred.uda.gpu.hbm.budget caps
    the device at --budget-gb and mapred.uda.gpu.merge.bytes at --merge-gb, so the task takes the GPU
    hybrid merge (direct RPQ key-range rounds over the fetched partitions; the reference's LPQ/RPQ,
    src/Merger/MergeManager.cc:202-288). The stream is validated natively (framing, key order, record
    checksum against the generated runs)."""
    import resource
    from uda_amd import native
    from uda_amd.bridge import UdaConsumer, UdaProvider
    from uda_amd.utils.datagen import TEXT
    from uda_amd.utils.mof import encode_partitions
    n = native()
    rows = int(args.gb * 1e9 / 100 / args.maps)
    prov = UdaProvider()
    total, want_sum = 0, 0
    for m in range(args.maps):  # one map at a time: the host holds the encoded MOFs, not the runs too
        parts = n.generate_runs("secondary", 1, 1, rows, 1000 + m)[0]
        want_sum = (want_sum + n.ifile_checksum(parts[0])[2]) & 0xFFFFFFFFFFFFFFFF
        data, index = encode_partitions(parts)
        total += len(data) - 2
        prov.add_mof_memory("job_hb", f"attempt_hb_m_{m:06d}_0", data, index)
        del parts
        if m % 8 == 7:  # progress (a GPU box takes a silent minute for a hung run)
            print(f"# hybrid_budget: {m + 1}/{args.maps} maps, {total / 1e9:.1f} GB", file=sys.stderr, flush=True)
    budget = int(args.budget_gb * 1e9)
    conf = {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.hbm.budget": budget,
            "mapred.uda.gpu.merge.bytes": int(args.merge_gb * 1e9), "mapred.uda.gpu.spill": "host"}
    c = UdaConsumer(args.maps, "job_hb", "attempt_hb_r_000000_0", TEXT, conf=conf, keep_records=False, validate=True)
    t0 = time.perf_counter()
    for m in range(args.maps):
        c.fetch("localhost", "job_hb", f"attempt_hb_m_{m:06d}_0", 0)
    while not c._done.wait(30):
        print(f"# hybrid_budget: merging, {time.perf_counter() - t0:.0f} s, "
              f"{c.validator.records if c.validator else 0} records delivered", file=sys.stderr, flush=True)
    c.wait(1)
    wall = time.perf_counter() - t0
    st = c.close()
    v = c.validator
    prov.close()
    hs = n.hbm_stats(0)
    out = {"config": "one NetMerger task over host MOFs, partition >> device budget (GPU hybrid)",
           "gb": round(total / 1e9, 3), "maps": args.maps, "budget_gb": args.budget_gb, "merge_gb": args.merge_gb,
           "ratio_partition_to_budget": round(total / budget, 2), "gbps": round(total / wall / 1e9, 3),
           "wall_s": round(wall, 2), "merge_path": st.get("merge_path"), "hybrid_direct": st.get("hybrid_direct"),
           "rpq_rounds": st.get("rpq_rounds"), "lpqs": st.get("lpqs"), "delivered_ok": st["bytes_delivered"] - 2 == total,
           "ledger_peak_gb": round(hs["peak"] / 1e9, 2), "device_peak_gb": round(hs["device_peak"] / 1e9, 2),
           "over_budget_bytes": hs["over"], "max_rss_gb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 1)}
    out["validation"] = {"records": v.records, "order_errors": v.order_errors, "framing_errors": v.framing_errors,
                         "eof": v.eof, "checksum_ok": v.checksum == want_sum}
    out["validated"] = bool(v.order_errors == 0 and v.framing_errors == 0 and v.eof and v.checksum == want_sum
                            and out["delivered_ok"])
    return out


def aio(args) -> dict:
    """AsyncIO read bandwidth vs a sequential pread loop (the reference's AIOHandler_test)."""
    from uda_amd import native
    path = os.path.join(args.dir, "uda_aio_bench.bin")
    size = int(args.gb * 1e9) // (1 << 20) * (1 << 20)
    out = {"config": "AIO microbenchmark (io_uring, O_DIRECT, 1 MiB blocks)", "gb": round(size / 1e9, 3)}
    for be in ("", "threadpool"):
        r = native().aio_bench(path, size, 1 << 20, 16, True, be)
        out[(r["backend"]) + "_mbps"] = round(r["aio_mbps"], 1)
        out[(r["backend"]) + "_streaming_mbps"] = round(r["aio_streaming_mbps"], 1)
        out["sequential_mbps"] = round(r["sequential_mbps"], 1)
        assert r["ok"]
    # the store loader's pattern: 32 files read round-robin in 16 MiB chunks, 16 in flight
    ib = native().aio_interleave_bench
    out["interleaved_32x16MiB_gbps"] = round(ib(args.dir, 32, size // 32, 16 << 20, 16), 2)
    out["interleaved_32x1MiB_d64_gbps"] = round(ib(args.dir, 32, size // 32, 1 << 20, 64), 2)
    out["interleaved_32x2MiB_d64_gbps"] = round(ib(args.dir, 32, size // 32, 2 << 20, 64), 2)
    out["interleaved_32x4MiB_d32_gbps"] = round(ib(args.dir, 32, size // 32, 4 << 20, 32), 2)
    out["interleaved_32x1MiB_d256_gbps"] = round(ib(args.dir, 32, size // 32, 1 << 20, 256), 2)
    return out


def spill(args) -> dict:
    import torch  # noqa: F401
    from uda_amd.models.terasort import TeraSortConfig, TeraSortShuffle
    from uda_amd.parallel.dist import DistContext
    cfg = TeraSortConfig(rows_per_gpu=int(args.gb * 1e9 / 104), maps_per_rank=args.maps, rounds=args.rounds,
                         store="host", validate=args.validate)
    job = TeraSortShuffle(DistContext(), cfg, device=0)
    job.setup()
    job.step()
    t0 = time.perf_counter()
    st = job.step()
    dt = time.perf_counter() - t0
    job.check(st)
    return {"config": "TeraSort with map outputs in pinned host DRAM (spill tier), 1 GPU",
            "gb": round(st["bytes_in"] / 1e9, 3), "wall_s": round(dt, 3),
            "shuffle_merge_gbps": round(st["bytes_in"] / dt / 1e9, 3),
            "breakdown_ms": {k: round(st[k], 1) for k in ("comm_ms", "merge_ms", "d2h_ms")}}


def radix(args) -> dict:
    """F8 map-side sort: one map output's records (uniform random 10-byte keys) sorted on the device by
    the LSD radix sort + gather (`csrc/gpu/radix.hip`); checked against numpy's stable lexsort."""
    import numpy as np
    from uda_amd import native
    n = int(args.gb * 1e9 / 104)
    rng = np.random.default_rng(11)
    r = np.empty((n, 104), dtype=np.uint8)
    r[:, 0], r[:, 1], r[:, 2], r[:, 13] = 0x0B, 0x5B, 0x0A, 0x5A
    r[:, 3:13] = rng.integers(0, 256, size=(n, 10), dtype=np.uint8)
    r[:, 14:] = ord("A") + (np.arange(90, dtype=np.uint8)[None, :] + r[:, 3:4]) % 26
    out, ms = native().gpu_sort_fixed(r, staged=True)  # the engine's layout: no copy aside
    keys = r[:, 3:13]
    order = np.lexsort(tuple(keys[:, j] for j in range(9, -1, -1)))  # stable, byte 0 most significant
    ok = out == r[order].tobytes()
    # HBM bytes the sort moves: key extract (104 read, 16 write), 10 passes of hist (16) + scatter (32),
    # and the gather (104 + 104 + 16 key read)
    moved = n * (104 + 16 + 10 * 48 + 224)
    return {"config": "F8 device radix sort of one map output (TeraSort records, 10-byte keys)",
            "records": n, "gb": round(n * 104 / 1e9, 3), "sort_ms": round(ms, 2),
            "mrecords_per_s": round(n / ms / 1e3, 1), "gbps_records": round(n * 104 / ms / 1e6, 1),
            "hbm_gbps_est": round(moved / ms / 1e6, 1), "matches_numpy_lexsort": bool(ok)}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("config", choices=["wordcount_loopback", "wordcount_tcp", "cpu_reference", "secondary_sort", "spill", "decode", "aio",
                                       "netmerger", "radix", "hybrid_budget"])
    ap.add_argument("--dir", default="/tmp")
    ap.add_argument("--codec", default="snappy", choices=["snappy", "lzo"])
    ap.add_argument("--gb", type=float, default=1.0)
    ap.add_argument("--maps", type=int, default=16)
    ap.add_argument("--reducers", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--validate", action="store_true")
    ap.add_argument("--budget-gb", type=float, default=10.0, help="hybrid_budget: mapred.uda.gpu.hbm.budget")
    ap.add_argument("--merge-gb", type=float, default=8.0, help="hybrid_budget: mapred.uda.gpu.merge.bytes")
    a = ap.parse_args()
    fn = globals()[a.config]
    out = fn(a)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
