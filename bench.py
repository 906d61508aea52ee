#!/usr/bin/env python3
"""Headline benchmark: TeraSort shuffle+merge GB/s, whole node (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W

One process per GPU. Under torchrun (RANK/LOCAL_RANK/WORLD_SIZE set) this process is one rank;
otherwise `--gpus N` (N > 1) starts the N rank processes itself (before anything touches the GPU)
with a 127.0.0.1 rendezvous, and rank 0 prints the result.

One step = the whole reduce-side shuffle of a TeraSort job: every GPU hosts `--reducers` reduce
tasks; each reducer receives its key range from every GPU's map outputs (RCCL all-to-all over
xGMI in key-range rounds), merges it on the GPU and its consumer thread receives the merged
records in <=1 MiB whole-record buffers (the `dataFromUda` contract, EOF marker included). The
consumer does the Java side's work on every buffer: copy into a 1 MiB KVBuf and walk the records
by their VInt lengths (J2CQueue); every step checks the parsed record count of every reducer.
Per-GPU data is fixed (weak scaling): --rows-per-gpu TeraGen rows (104-byte IFile records) per
GPU; the default 1.25e9 rows/GPU makes N=8 the 1 TB TeraSort config (N=1 moves 130 GB).

After the timed steps one more (untimed) step runs with the device-side validation on: key order
per reducer, record checksum against the generated data, and (N > 1) per-slice checksums of what
every peer sent. "validated": true means that step passed.

value = total partition bytes delivered on all GPUs / time per step (GB = 1e9 bytes).
Data is synthetic (TeraGen-shaped keys/values generated in HBM; see uda_amd/models/terasort.py).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows-per-gpu", type=int, default=1_250_000_000)
    ap.add_argument("--maps-per-gpu", type=int, default=32)
    ap.add_argument("--reducers", type=int, default=16,
                    help="reduce tasks per GPU (each with its own consumer thread; 16 leaves the host side "
                         "headroom when 8 GPUs stream into one node's DRAM)")
    ap.add_argument("--rounds", type=int, default=16, help="key cells per reducer = shuffle rounds per step")
    ap.add_argument("--d2h", choices=("sdma", "hip"), default="sdma",
                    help="delivery copies: explicit SDMA engines (default) or hipMemcpyAsync")
    ap.add_argument("--d2h-piece-mb", type=int, default=128)
    ap.add_argument("--pinned-slots", type=int, default=16)
    ap.add_argument("--d2h-engines", type=int, default=1)
    ap.add_argument("--replan", action="store_true",
                    help="recompute the cell splits (and re-exchange the slice counts) inside every timed "
                         "step instead of reusing the setup-time plan")
    ap.add_argument("--api-host-mofs", action="store_true",
                    help="--api: map outputs registered from host memory (fetched as bytes, staged to HBM)")
    ap.add_argument("--api-fetch", choices=("device", "host", "auto"), default=None,
                    help="--api: mapred.uda.gpu.fetch of the reduce tasks (default: device, host with --api-host-mofs)")
    ap.add_argument("--api-gpu-slots", type=int, default=-1,
                    help="--api: mapred.uda.gpu.max.concurrent.merges (staged GPU merges admitted at once; 0: all; "
                         "default: 6 with --api-host-mofs, else the native default, 0 = off)")
    ap.add_argument("--api-provider-workers", type=int, default=-1,
                    help="--api: mapred.uda.provider.workers of the MOFSupplier (default 8)")
    ap.add_argument("--one-gpu", action="store_true",
                    help="N ranks, every rank on GPU 0: rehearsal of the multi-process path on a one-GPU machine "
                         "(--exchange ipc or --api; RCCL refuses two ranks on one GPU)")
    ap.add_argument("--exchange", choices=("ipc", "rccl"), default="ipc",
                    help="N > 1: all-to-all-v backend of the shuffle rounds: 'ipc' (node-local shared-memory "
                         "control plane, pull copies from the peers' HBM mapped over hipIpc; default) or 'rccl' "
                         "(grouped ncclSend/ncclRecv)")
    ap.add_argument("--map-sort", action=argparse.BooleanOptionalAction, default=True,
                    help="setup generates unsorted TeraGen map input (uniform random keys) and sorts every "
                         "map-output partition on the device (F8 radix sort), like a map task's sort before "
                         "its spill (default); --no-map-sort generates the sorted runs directly")
    ap.add_argument("--store", choices=("hbm", "host", "disk"), default="hbm",
                    help="map-output store: HBM (default), pinned host DRAM, or MOF files on --local-dirs")
    ap.add_argument("--local-dirs", default="/tmp", help="--store disk: comma-separated directories")
    ap.add_argument("--max-round-gb", type=float, default=0.0,
                    help="bound the HBM staging per round (raises --rounds so a round is at most this size)")
    ap.add_argument("--device-only", action="store_true",
                    help="ablation: stop after the device merge (no host delivery); not the headline")
    ap.add_argument("--no-validate", action="store_true", help="skip the final validated step")
    ap.add_argument("--sink", choices=("j2c", "none"), default="j2c",
                    help="ablation: 'none' drops delivered buffers unread (measures the copy path alone)")
    ap.add_argument("--api", action="store_true",
                    help="drive the shuffle only through the UdaBridge C ABI (uda_start/INIT/FETCH/dataFromUda) "
                         "with HBM-resident MOFs: one NetMerger handle per reduce task (1 GPU)")
    ap.add_argument("--round-mb", type=int, default=2048, help="--api: device merge round size per reduce task")
    ap.add_argument("--workload", choices=("terasort", "secondary"), default="terasort",
                    help="--api: 'secondary' = BASELINE config #5: variable-length Text keys with long common "
                         "prefixes, --skew of every map's records to reduce task 0, merged on the device in "
                         "key-range rounds of --round-mb")
    ap.add_argument("--skew", type=float, default=0.6, help="--api --workload secondary: share of reduce task 0")
    ap.add_argument("--api-codec", choices=("snappy", "lzo"), default=None,
                    help="--api: map outputs block-compressed (256 KiB blocks) and registered in HBM; reduce tasks "
                         "decode on the device straight from the descriptors (F6)")
    ap.add_argument("--mof-dir", default="",
                    help="--api: write every map output as a file.out under this directory; the provider finds "
                         "them through getPathUda (Hadoop-written MOFs) and serves them from its HBM store. "
                         "With --node: the documented deployment end to end (map phase writes the files, provider "
                         "front end + node daemon with default configuration, reduce tasks with no mapred.uda.* key)")
    ap.add_argument("--provider-hbm-gb", type=float, default=-1.0,
                    help="--api --mof-dir: mapred.uda.provider.hbm.bytes in GB (default: 1.25x the MOF bytes; "
                         "0 = store off: descriptor fetches are declined and reducers fetch bytes)")
    ap.add_argument("--node", action="store_true",
                    help="--api: the node shape: this process is the node's MOFSupplier (map outputs in its HBM, TCP) "
                         "and every step is a wave of --reducers reduce tasks, each a fresh process "
                         "(uda_amd/bin/uda_reduce_task: uda_start, INIT, FETCHes, dataFromUda into a J2C consumer), "
                         "as YARN runs one JVM per reduce task; value includes the processes' start")
    ap.add_argument("--node-gap", type=float, default=0.0,
                    help="--node: seconds between a wave's INITs and its FETCHes (reduce slow-start: the tasks start "
                         "while the maps still run); 0 = the tasks start when every map output is there")
    ap.add_argument("--node-service", action=argparse.BooleanOptionalAction, default=True,
                    help="--node: the supplier process is also the node's merge service (every reduce task process "
                         "is a thin client whose NetMerger runs in the service: one GPU context, warm pools and "
                         "the HBM store in one process; mapred.uda.gpu.merge.service; the recommended deployment). "
                         "--no-node-service: every task merges in its own fresh process")
    ap.add_argument("--node-slots", type=int, default=15,
                    help="--node: reduce task processes running at once (YARN containers of the node); the one-GPU "
                         "box allows 16 GPU processes, the provider is one of them")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--launch-selftest", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str]) -> int:
    """Start one process per GPU (RANK/LOCAL_RANK/WORLD_SIZE in their env); return the worst rc."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env, cwd=ROOT))
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        failed = [rc for rc in rcs if rc not in (None, 0)]
        if failed:  # one rank died: the others would wait for it in a collective
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        time.sleep(0.2)
    return max(abs(rc) for rc in rcs)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, argv)
    if args.launch_selftest:  # launcher check (CPU tests): report the rank environment, touch no GPU
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                          "MASTER_PORT")}), flush=True)
        return 0

    import torch  # noqa: F401  (loads the HIP runtime before the native extension)

    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from uda_amd import native
    from uda_amd.models.terasort import RECORD_BYTES, TeraSortConfig, TeraSortShuffle
    from uda_amd.parallel.dist import init_from_env

    ctx = init_from_env()
    if ctx.world != args.gpus:
        print(f"bench: --gpus {args.gpus} but the launcher started {ctx.world} rank(s)", file=sys.stderr)
        return 2
    if args.api and args.node:  # every GPU call in native processes (this one only orchestrates)
        return run_node_files(args, ctx) if args.mof_dir else run_node(args, ctx)
    if args.api:
        torch.cuda.set_device(0 if args.one_gpu else ctx.local_rank)
        return run_api(args, ctx)
    if args.one_gpu and ctx.world > 1 and args.exchange == "rccl":
        print("bench: --one-gpu needs --exchange ipc (RCCL refuses two ranks on one GPU)", file=sys.stderr)
        return 2
    device = 0 if args.one_gpu else ctx.local_rank
    torch.cuda.set_device(device)

    rounds = args.rounds
    if args.max_round_gb > 0:
        rounds = max(rounds, -(-int(args.rows_per_gpu * RECORD_BYTES) // int(args.max_round_gb * 1e9)))
    cfg = TeraSortConfig(rows_per_gpu=args.rows_per_gpu, maps_per_rank=args.maps_per_gpu,
                         rounds=rounds, reducers=args.reducers, d2h=args.d2h, store=args.store,
                         local_dirs=args.local_dirs,
                         d2h_piece_bytes=args.d2h_piece_mb << 20, pinned_slots=args.pinned_slots,
                         d2h_engines=args.d2h_engines, deliver_host=not args.device_only,
                         replan=args.replan, map_sort=args.map_sort, exchange=args.exchange)
    job = TeraSortShuffle(ctx, cfg, device=device)
    t_setup = time.perf_counter()
    job.setup()
    if args.sink == "none":
        job.drop_sink()
    t_setup = time.perf_counter() - t_setup
    if ctx.rank == 0:
        print(f"# setup {t_setup:.1f}s cpus={len(os.sched_getaffinity(0))} {job.setup_s} "
              f"store={job.job.store_bytes/1e9:.1f}GB "
              f"max_round_records={job.job.max_round_records} exchange={job.job.exchange_name} "
              f"store={job.job.store_name} "
              f"delivery={job.job.delivery_name}"
              + (f" map_sort_ms={job.job.map_sort_ms:.1f}" if args.map_sort else ""), file=sys.stderr, flush=True)

    for i in range(args.warmup):
        st = job.step()
        job.check(st)
        if args.verbose and ctx.rank == 0:
            print(f"# warmup {i}: {json.dumps(st)}", file=sys.stderr, flush=True)

    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        stats.append(job.step())
    torch.cuda.synchronize()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = ctx.max_float(elapsed)
    for st in stats:
        job.check(st)  # consumer record counts / framing / EOF of every timed step

    validated = None
    exchange_errors = None
    if not args.no_validate:
        vst = job.step(validate=True)
        job.check(vst)  # raises on order / checksum / exchange-checksum errors
        ok = ctx.all_gather_object(int(vst["exchange_errors"]))
        exchange_errors = sum(ok)
        validated = exchange_errors == 0
        if args.verbose and ctx.rank == 0:
            print(f"# validated step: {json.dumps(vst)}", file=sys.stderr, flush=True)

    bytes_per_gpu = stats[0]["bytes_in"]
    total_bytes = sum(ctx.all_gather_object(bytes_per_gpu))
    details = ctx.all_gather_object(rank_detail(args, ctx, job, device, stats))
    sent = ctx.all_gather_object(int(sum(s["bytes_sent"] for s in stats) // max(1, len(stats))))
    ms_per_step = elapsed * 1000.0 / max(1, args.steps)
    gbps = total_bytes / (ms_per_step / 1000.0) / 1e9
    mean = lambda k: sum(s[k] for s in stats) / len(stats)  # noqa: E731
    comm_ranks = job.job.comm_ranks if ctx.world > 1 else None
    if ctx.rank == 0:
        out = {
            "metric": "TeraSort shuffle+merge GB/s whole-node",
            "value": round(gbps, 3),
            "unit": "GB/s",
            "n_gpus": 1 if args.one_gpu else ctx.world,
            "ranks": ctx.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bytes",
            "data": ("synthetic TeraGen-shaped (uniform random 10B keys, 90B values, 104B IFile records "
                     "generated in HBM; map outputs sorted by the device radix sort at setup)") if args.map_sort else
                    "synthetic TeraGen-shaped (10B key/90B value, 104B IFile records generated in HBM)",
            "map_sort_ms": round(job.job.map_sort_ms, 1) if args.map_sort else None,
            "breakdown_note": "comm/merge: device-event spans per round; d2h: summed piece latency; "
                              "wait_out: merge waiting for a free output slot (delivery-bound)",
            "config": {
                "model": "terasort",
                "global_batch": int(args.rows_per_gpu) * ctx.world,
                "seq_len": RECORD_BYTES,
                "parallelism": f"dp{ctx.world}" + (" (ranks share GPU 0: rehearsal)" if args.one_gpu and ctx.world > 1
                                                    else ""),
                "rows_per_gpu": args.rows_per_gpu,
                "total_rows": args.rows_per_gpu * ctx.world,
                "maps_per_gpu": args.maps_per_gpu,
                "reducers_per_gpu": args.reducers,
                "rounds": rounds,
                "store": job.job.store_name,
                "shuffle": job.job.exchange_name if ctx.world > 1 else "local (single GPU, no all-to-all)",
                "delivery": "device-only (ablation)" if args.device_only else
                            f"{job.job.delivery_name} -> buffers dropped unread (ablation)" if args.sink == "none" else
                            f"{job.job.delivery_name} -> per-reducer J2C consumer (KVBuf memcpy + VInt walk), <=1MiB buffers",
            },
            "reduce_wall_clock_s": round(ms_per_step / 1000.0, 3),
            "teragen_gbps": round(gbps * 100 / RECORD_BYTES, 3),
            "exchange": job.job.exchange_name if ctx.world > 1 else None,
            "comm_ranks": comm_ranks,
            "bytes_sent_per_rank": sent,
            "breakdown_ms_rank0": {k: round(mean(k), 2) for k in ("plan_ms", "comm_ms", "merge_ms", "d2h_ms",
                                                                  "wait_out_ms", "stage_ms")},
            "replan_in_step": bool(args.replan),
            "merge_passes": stats[0]["merge_passes"],
            "buffers_per_step": stats[0]["buffers"],
            "validated": validated,
            "exchange_errors": exchange_errors,
            "ipc_fallback": getattr(job, "ipc_fallback", None),
            "hbm_over_budget_bytes": int(native().hbm_stats(device)["over"]),
            "reference_envelope_gbps_per_node": 5.0,
            # self-diagnosis of a multi-GPU record: where every rank's threads, rings and bytes went
            "peer_access": native().peer_access_matrix(),
            "ipc_preflight": (None if ctx.world == 1 or args.exchange != "ipc" else
                              "skipped (UDA_IPC_PREFLIGHT=0)" if os.environ.get("UDA_IPC_PREFLIGHT", "1") == "0" else
                              "passed" if getattr(job, "ipc_fallback", None) is None else "failed"),
            "ranks_detail": details,
        }
        out["record_complete"] = record_problems(out) == []
        print(json.dumps(out), flush=True)
    ctx.close()
    return 0


RANK_DETAIL_KEYS = {"rank": int, "device": int, "numa_node": int, "consumer_cpus": str, "delivery": str,
                    "exchange_why": str, "peer_send_bytes": list, "round_comm_ms": list, "round_merge_ms": list,
                    "wall_ms": float, "comm_ms": float, "merge_ms": float, "d2h_ms": float, "wait_out_ms": float,
                    "bytes_in": int}


def record_problems(out: dict) -> list[str]:
    """What a multi-GPU record lacks to be diagnosable: one ranks_detail entry per rank with every field
    of RANK_DETAIL_KEYS, per-peer bytes for every peer, a per-round span for every round, and the
    peer-access matrix."""
    probs = []
    det = out.get("ranks_detail") or []
    if len(det) != out.get("ranks"):
        probs.append(f"ranks_detail has {len(det)} entries for {out.get('ranks')} ranks")
    rounds = (out.get("config") or {}).get("rounds")
    for d in det:
        for k, t in RANK_DETAIL_KEYS.items():
            v = d.get(k)
            if v is None or not isinstance(v, (int, float) if t is float else t):
                probs.append(f"rank {d.get('rank')}: {k} missing or not {t.__name__}")
        if len(d.get("peer_send_bytes") or []) != out.get("ranks"):
            probs.append(f"rank {d.get('rank')}: peer_send_bytes is not per peer")
        if rounds and len(d.get("round_merge_ms") or []) != rounds:
            probs.append(f"rank {d.get('rank')}: round_merge_ms is not per round")
    if not isinstance(out.get("peer_access"), list):
        probs.append("peer_access matrix missing")
    return probs


def rank_detail(args, ctx, job, device, stats) -> dict:
    """One rank's placement and timings for the bench record (rank 0 gathers every rank's): GPU -> NUMA
    node -> consumer CPU slice, delivery ring / SDMA engines, exchange backend and why, bytes per peer,
    per-round exchange and merge spans, and the delivery-side waits (d2h, wait_out)."""
    from uda_amd import native
    n = len(stats)
    mean = lambda k: round(sum(s[k] for s in stats) / max(1, n), 2)  # noqa: E731
    per_round = lambda k: [round(sum(s[k][q] for s in stats) / max(1, n), 2)  # noqa: E731
                           for q in range(len(stats[0].get(k, [])))]
    if ctx.world == 1:
        why = "single GPU: no all-to-all"
    elif getattr(job, "ipc_fallback", None):
        why = f"IPC preflight failed, RCCL instead: {job.ipc_fallback}"
    else:
        why = f"--exchange {args.exchange}" + (" (default)" if args.exchange == "ipc" else "")
    d = {"rank": ctx.rank, "device": device}
    d.update(native().device_placement(device))
    d.update({
        "delivery": job.job.delivery_name,  # SDMA engines for D2H / H2D and the pinned ring's NUMA pages
        "exchange": job.job.exchange_name if ctx.world > 1 else None,
        "exchange_why": why,
        "peer_send_bytes": list(job.job.peer_send_bytes()),
        "round_comm_ms": per_round("round_comm_ms"),
        "round_merge_ms": per_round("round_merge_ms"),
        "wall_ms": mean("wall_ms"),
        "comm_ms": mean("comm_ms"),
        "merge_ms": mean("merge_ms"),
        "d2h_ms": mean("d2h_ms"),
        "wait_out_ms": mean("wait_out_ms"),
        "bytes_in": stats[0]["bytes_in"],
    })
    return d


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def run_node(args, ctx) -> int:
    """The node shape of a Hadoop job on one GPU: the node's MOFSupplier is a process of its own
    (uda_amd/bin/uda_mof_supplier, the NodeManager aux service, MOFSupplierMain.cc:87-143) holding the
    maps' outputs in its HBM and serving them over TCP; a step is a wave of reduce tasks, each started
    as a fresh process (uda_amd/bin/uda_reduce_task; UdaBridge.cc:187-263, NetMergerMain.cc:44-77: one
    NetMerger per ReduceTask JVM) that INITs, FETCHes its partition of every map as device descriptors
    (the supplier's HBM mapped over hipIpc), merges on the GPU and walks every delivered buffer. This
    process only orchestrates (no GPU call), so every process on the GPU uses the system HIP runtime,
    as on a Hadoop node. value = record bytes delivered / wall time of the wave, process starts included."""
    import statistics
    import subprocess as sp

    if ctx.world != 1:
        print("bench: --node runs one supplier process per node (--gpus 1)", file=sys.stderr)
        return 2
    bindir = os.path.join(ROOT, "uda_amd", "bin")
    exe, sup = os.path.join(bindir, "uda_reduce_task"), os.path.join(bindir, "uda_mof_supplier")
    for x in (exe, sup):
        if not os.access(x, os.X_OK):
            print(f"bench: {x} is missing; build with python tools/build.py", file=sys.stderr)
            return 2
    R = args.reducers
    logdir = os.path.join(ROOT, "gpurun_out") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else "/tmp"
    errlog = open(os.path.join(logdir, "node_tasks.err"), "a")
    args.service_path = f"/tmp/uda-merge-{os.getpid()}.sock" if args.node_service else ""
    supplier = sp.Popen([sup, "device=0", f"service={args.service_path}", f"maps={args.maps_per_gpu}", f"reducers={R}",
                         f"records_per_map={max(1, args.rows_per_gpu // args.maps_per_gpu)}",
                         f"round_bytes={args.round_mb << 20}", f"workload={args.workload}", f"skew={args.skew}",
                         f"codec={args.api_codec or ''}", f"port={_free_port()}", "bind=127.0.0.1",
                         f"workers={args.api_provider_workers}"],
                        stdin=sp.PIPE, stdout=sp.PIPE, stderr=errlog, text=True, cwd=ROOT)
    try:
        return _node_waves(args, supplier, exe, errlog, statistics, sp)
    finally:
        if supplier.poll() is None:
            try:
                supplier.stdin.write("exit\n")
                supplier.stdin.flush()
                supplier.wait(60)
            except (OSError, sp.TimeoutExpired):
                supplier.kill()
                supplier.wait()


def _node_waves(args, supplier, exe, errlog, statistics, sp) -> int:
    t = time.perf_counter()
    first = supplier.stdout.readline()
    info = json.loads(first) if first.strip() else {"error": f"supplier exited rc={supplier.poll()}"}
    if "error" in info:
        raise RuntimeError(f"MOF supplier failed: {info['error']}")
    R, port = args.reducers, info["port"]
    print(f"# node setup {time.perf_counter() - t:.1f}s store={info['store_bytes'] / 1e9:.1f}GB supplier pid "
          f"{supplier.pid} port {port}, {R} reduce task processes per wave, {args.node_slots} at once",
          file=sys.stderr, flush=True)
    conf = {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.fetch": "device", "mapred.uda.transport": "tcp",
            "mapred.uda.gpu.device": "auto", "mapred.uda.gpu.round.bytes": str(args.round_mb << 20),
            "mapred.uda.gpu.merge.service": args.service_path or "off"}
    for kv in filter(None, os.environ.get("UDA_API_CONF", "").split(",")):
        k, _, v = kv.partition("=")
        conf[k] = v
    warm, stats, validated = _run_waves(args, port, info["commands"], info["expected"], exe, errlog, conf, sp,
                                        statistics)
    supplier.stdin.write("stats\n")
    supplier.stdin.flush()
    provider = json.loads(supplier.stdout.readline())
    out = _node_result(args, stats, warm, validated, provider)
    out["config"]["shuffle"] = (
        "node shape: one MOFSupplier process (uda_mof_supplier: map outputs in its HBM, TCP control) + one fresh "
        "process per reduce task (uda_reduce_task: INIT/FETCH/dataFromUda), " +
        ("NetMergers hosted by the supplier's merge service, merged buffers read in place from its shared pinned "
         "rings" if args.service_path else "descriptors mapped over hipIpc"))
    out["node"]["merge_service"] = bool(args.service_path)
    print(json.dumps(out), flush=True)
    return 0


def _run_waves(args, port, cmds, expected, exe, errlog, conf, sp, statistics):
    """Warmup waves, timed waves and the validated wave of R fresh reduce task processes."""
    R = args.reducers
    start = ["-w", "256", "-r", str(port), "-a", "1", "-m", "1", "-g", "/tmp", "-s", "1024"]

    def wave(validate: bool) -> dict:
        t0 = time.perf_counter()
        todo, running, out = list(range(R)), {}, {}
        t_fetch = None

        def launch(r):
            argv = [exe]
            for k, v in conf.items():
                argv += ["-D", f"{k}={v}"]
            argv += ["--expect", str(expected[r])] + (["--check-order"] if validate else []) + ["--"] + start
            p = sp.Popen(argv, stdin=sp.PIPE, stdout=sp.PIPE, stderr=errlog, text=True, cwd=ROOT)
            p.stdin.write(cmds[r][0] + "\n")  # INIT: the task starts (prewarm) while maps may still run
            p.stdin.flush()
            return p

        def fetch(p, r):
            p.stdin.write("\n".join(cmds[r][1:]) + "\n")
            p.stdin.close()

        while todo or running:
            while todo and len(running) < args.node_slots:
                r = todo.pop(0)
                running[r] = launch(r)
                if t_fetch is not None:  # a later container: its maps are long done
                    fetch(running[r], r)
            if t_fetch is None:
                time.sleep(args.node_gap)
                t_fetch = time.perf_counter()
                for r, p in running.items():
                    fetch(p, r)
            for r, p in list(running.items()):
                if p.poll() is not None:
                    line = p.stdout.read().strip().splitlines()
                    res = json.loads(line[-1]) if line else {"error": "no output"}
                    if p.returncode != 0 or res.get("error"):
                        t = res.get("task") or {}
                        print(f"# failed reduce task {r}: " + json.dumps({k: t.get(k) for k in (
                            "merge_path", "device_descriptors", "host_fetched_bytes", "maps_fetched", "bytes_fetched",
                            "records", "bytes_delivered", "unmapped_descriptors", "merge_service", "rpq_rounds")}),
                              file=sys.stderr, flush=True)
                        raise RuntimeError(f"reduce task {r} (pid {p.pid}) failed rc={p.returncode}: {res.get('error')}")
                    out[r] = res
                    del running[r]
            time.sleep(0.002)
        t1 = time.perf_counter()
        med = lambda k: round(statistics.median(o[k] for o in out.values()), 1)  # noqa: E731
        # per task, ms after the wave's first exec (CLOCK_BOOTTIME, the tasks' own clock): exec, first
        # FETCH, first dataFromUda, EOF walked, process end
        t_base = min(o["t_exec_boot_ms"] for o in out.values())
        timeline = []
        for r in sorted(out):
            o = out[r]
            ff = o["t_exec_boot_ms"] + o["first_fetch_ms"]
            eof = o["t_end_boot_ms"] - o["exit_ms"]
            timeline.append([round(x - t_base) for x in (o["t_exec_boot_ms"], ff, ff + o["fetch_to_first_data_ms"],
                                                         eof, o["t_end_boot_ms"])])
        # which path each task's partitions took: device descriptors of the provider's HBM store, or bytes
        # (declined by a full store, fetched over TCP and staged); per-path task times
        paths = {}
        for o in out.values():
            t = o["task"]
            kind = "bytes_and_descriptors" if t.get("host_fetched_bytes", 0) > 0 and t.get("device_descriptors", 0) > 0 \
                else "bytes_only" if t.get("host_fetched_bytes", 0) > 0 else "descriptors_only"
            pth = paths.setdefault(kind, {"tasks": 0, "fetch_to_eof_ms": []})
            pth["tasks"] += 1
            pth["fetch_to_eof_ms"].append(o["fetch_to_eof_ms"])
        for pth in paths.values():
            v = sorted(pth.pop("fetch_to_eof_ms"))
            pth["fetch_to_eof_ms_median"] = round(v[len(v) // 2], 1)
            pth["fetch_to_eof_ms_max"] = round(v[-1], 1)
        split = {"descriptors": sum(int(o["task"].get("device_descriptors", 0)) for o in out.values()),
                 "bytes_fetched_as_bytes": sum(int(o["task"].get("host_fetched_bytes", 0)) for o in out.values()),
                 "of_which_read_from_mof_files": sum(int(o["task"].get("local_read_bytes", 0)) for o in out.values()),
                 "hbm_wait_ms_max": round(max(float(o["task"].get("hbm_wait_ms", 0)) for o in out.values()), 1),
                 "paths": paths}
        return {"wall_ms": (t1 - t0) * 1e3, "from_fetch_ms": (t1 - t_fetch) * 1e3, "timeline": timeline,
                "fetch_split": split,
                "t_base_boot_ms": t_base,
                "bytes": sum(o["bytes"] for o in out.values()), "records": sum(o["records"] for o in out.values()),
                "order_errors": sum(o["order_errors"] for o in out.values()),
                "task_ms_median": {k: med(k) for k in ("exec_to_main_ms", "start_ms", "init_ms",
                                                       "fetch_to_first_data_ms", "fetch_to_eof_ms", "exit_ms")},
                "task0": out[0]["task"]}

    warm = []
    for i in range(args.warmup):
        warm.append(wave(False))
        if args.verbose:
            print(f"# warmup {i}: {json.dumps(warm[-1])}", file=sys.stderr, flush=True)
    stats = [wave(False) for _ in range(args.steps)]
    validated = None
    if not args.no_validate:
        validated = wave(True)["order_errors"] == 0
    return warm, stats, validated


def _node_result(args, stats, warm, validated, provider) -> dict:
    R = args.reducers
    ms = sum(s["wall_ms"] for s in stats) / len(stats)
    fetch_ms = sum(s["from_fetch_ms"] for s in stats) / len(stats)
    nbytes = stats[0]["bytes"]
    return {
        "metric": "TeraSort shuffle+merge GB/s whole-node",
        "value": round(nbytes / ms / 1e6, 3),
        "unit": "GB/s",
        "n_gpus": 1,
        "ranks": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bytes",
        "data": "synthetic TeraGen-shaped (10B key/90B value, 104B IFile records generated in HBM)"
                if args.workload == "terasort" else f"synthetic secondary-sort map outputs, {args.skew:.0%} skew",
        "config": {"model": "terasort" if args.workload == "terasort" else "secondary-sort",
                   "global_batch": int(stats[0]["records"]), "seq_len": 104, "parallelism": "dp1",
                   "rows_per_gpu": args.rows_per_gpu, "maps_per_gpu": args.maps_per_gpu, "reducers_per_gpu": R,
                   "shuffle": "",
                   "delivery": "dataFromUda -> J2C consumer (KVBuf memcpy + VInt walk) in each task process"},
        "node": {"slots": args.node_slots, "gap_s": args.node_gap,
                 "gbps_from_fetch": round(nbytes / fetch_ms / 1e6, 3), "from_fetch_ms": round(fetch_ms, 1),
                 "warmup_step_ms": [round(st["wall_ms"], 1) for st in warm],
                 "step_ms": [round(st["wall_ms"], 1) for st in stats],
                 "task_ms_median": stats[-1]["task_ms_median"],
                 "timeline_ms": {"columns": ["exec", "first_fetch", "first_data", "eof", "end"],
                                 "tasks": stats[-1]["timeline"]}},
        "task0_stats": stats[-1]["task0"],
        "provider": provider,
        "validated": validated,
        "reference_envelope_gbps_per_node": 5.0,
    }


def _check_space(path: str, need: int) -> None:
    """The map outputs must fit the file system they are written to (a GPU box's /tmp is ~79 GB)."""
    os.makedirs(path, exist_ok=True)
    st = os.statvfs(path)
    free = st.f_bavail * st.f_frsize
    if free < need * 1.02:
        raise SystemExit(f"bench: {need / 1e9:.1f} GB of MOF files do not fit {path} ({free / 1e9:.1f} GB free); "
                         "lower --rows-per-gpu or point --mof-dir elsewhere")


def run_node_files(args, ctx) -> int:
    """The deployment as documented, end to end, on one GPU node: Hadoop-written map output files, the
    provider front end (the NodeManager's aux service: uda_mof_supplier mode=frontend, getPathUda over
    <mof-dir>/<map attempt>/file.out + file.out.index, no GPU call) with the library's defaults -- which
    start the node daemon holding the HBM store (files loaded on first touch) and the merge service -- and
    waves of fresh reduce task processes with NO mapred.uda.* key: each is hosted by the daemon's merge
    service, fetches its partitions as descriptors of the store and reads the merged buffers from its
    shared pinned rings. The first wave includes reading every MOF file from disk (a job reads each map
    output once): first_step_gbps; later waves merge from the store."""
    import shutil
    import statistics
    import subprocess as sp

    if ctx.world != 1:
        print("bench: --node runs one provider per node (--gpus 1)", file=sys.stderr)
        return 2
    if os.environ.get("UDA_API_CONF"):
        print("bench: --node --mof-dir measures the default configuration: unset UDA_API_CONF", file=sys.stderr)
        return 2
    bindir = os.path.join(ROOT, "uda_amd", "bin")
    exe, sup = os.path.join(bindir, "uda_reduce_task"), os.path.join(bindir, "uda_mof_supplier")
    R = args.reducers
    logdir = os.path.join(ROOT, "gpurun_out") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else "/tmp"
    errlog = open(os.path.join(logdir, "node_tasks.err"), "a")
    _check_space(args.mof_dir, args.rows_per_gpu * 104)  # TeraSort IFile records
    mof_dir = os.path.join(args.mof_dir, f"uda-node-{os.getpid()}")
    os.makedirs(mof_dir, exist_ok=True)
    frontend = None
    try:
        t = time.perf_counter()
        g = sp.run([sup, "mode=mapgen", f"mof_dir={mof_dir}", "device=0", f"maps={args.maps_per_gpu}",
                    f"reducers={R}", f"records_per_map={max(1, args.rows_per_gpu // args.maps_per_gpu)}",
                    f"workload={args.workload}", f"skew={args.skew}"],
                   stdout=sp.PIPE, stderr=errlog, text=True, cwd=ROOT, timeout=1800)
        lines = g.stdout.strip().splitlines()
        job = json.loads(lines[-1]) if lines else {"error": f"map phase exited rc={g.returncode}"}
        if g.returncode != 0 or "error" in job:
            raise RuntimeError(f"map phase failed: {job.get('error')}")
        t_map = time.perf_counter() - t
        port = _free_port()
        t = time.perf_counter()
        fe_conf = []
        if args.provider_hbm_gb >= 0:  # a store smaller than the map outputs: the mixed regime
            fe_conf.append(f"-Dmapred.uda.provider.hbm.bytes={int(args.provider_hbm_gb * 1e9)}")
        frontend = sp.Popen([sup, "mode=frontend", f"mof_dir={mof_dir}", f"port={port}"] + fe_conf, stdin=sp.PIPE,
                            stdout=sp.PIPE, stderr=errlog, text=True, cwd=ROOT,
                            env=dict(os.environ, UDA_DAEMON_LOG=os.path.join(logdir, "node_daemon.err")))
        first = frontend.stdout.readline()
        info = json.loads(first) if first.strip() else {"error": f"front end exited rc={frontend.poll()}"}
        if "error" in info:
            raise RuntimeError(f"provider front end failed: {info['error']}")
        # a NodeManager is up long before its first reduce task: wait for the node daemon (HBM store, merge
        # service) and its first-wave prewarm, as a job would find them
        t_ready = time.perf_counter()
        while True:
            frontend.stdin.write("stats\n")
            frontend.stdin.flush()
            hs = json.loads(frontend.stdout.readline()).get("hbm_store", {})
            if (hs.get("daemon", {}).get("ready") and hs.get("prewarm", {}).get("done", True)) or \
                    time.perf_counter() - t_ready > 120:
                break
            time.sleep(0.2)
        node_ready_s = time.perf_counter() - t
        daemon = dict(hs.get("daemon", {}), prewarm=hs.get("prewarm"))
        print(f"# node files: map phase {t_map:.1f}s ({job['store_bytes'] / 1e9:.1f} GB in {args.maps_per_gpu} "
              f"file.out), front end up in {time.perf_counter() - t:.1f}s, node daemon {daemon}", file=sys.stderr,
              flush=True)
        try:
            warm, stats, validated = _run_waves(args, port, job["commands"], job["expected"], exe, errlog, {}, sp,
                                                statistics)
        except RuntimeError as e:  # say whether the provider front end is still there
            rc = frontend.poll()
            how = "running" if rc is None else f"exited rc={rc}" + (f" (signal {-rc})" if rc < 0 else "")
            raise RuntimeError(f"{e}; provider front end pid {frontend.pid} {how}") from None
        frontend.stdin.write("stats\n")
        frontend.stdin.flush()
        provider = json.loads(frontend.stdout.readline())
        out = _node_result(args, stats, warm, validated, provider)
        out["config"]["shuffle"] = (
            "the documented deployment: Hadoop-layout MOF files -> provider front end (getPathUda, defaults) -> "
            "node daemon (HBM store, merge service) -> fresh reduce task processes with no mapred.uda.* keys")
        waves = warm + stats
        out["first_wave"] = {"timeline_ms": waves[0]["timeline"], "task_ms_median": waves[0]["task_ms_median"],
                             "task0": waves[0]["task0"]}
        hs = provider.get("hbm_store", {})
        if hs.get("first_miss_boot_ms"):  # the store's loads on the first wave's timeline (same clock)
            out["first_wave"]["store_ms"] = {k: round(hs[k + "_boot_ms"] - waves[0]["t_base_boot_ms"])
                                             for k in ("first_miss", "first_read", "last_landed")}
            if provider.get("first_descriptor_request_boot_ms"):  # the front end's first descriptor FETCH
                out["first_wave"]["store_ms"]["front_end_first_request"] = round(
                    provider["first_descriptor_request_boot_ms"] - waves[0]["t_base_boot_ms"])
        out["first_step_ms"] = round(waves[0]["wall_ms"], 1)
        out["first_step_gbps"] = round(waves[0]["bytes"] / waves[0]["wall_ms"] / 1e6, 3)
        out["mof_files_gb"] = round(job["store_bytes"] / 1e9, 2)
        out["conf_keys"] = 0
        out["node_ready_s"] = round(node_ready_s, 2)
        out["daemon_prewarm"] = daemon.get("prewarm")
        out["task0_hosted"] = bool(stats[-1]["task0"].get("merge_service"))
        out["provider_hbm_gb"] = args.provider_hbm_gb if args.provider_hbm_gb >= 0 else "default"
        out["fetch_split_first_step"] = waves[0]["fetch_split"]
        out["fetch_split_last_step"] = stats[-1]["fetch_split"]
        out["step_gbps"] = [round(w["bytes"] / w["wall_ms"] / 1e6, 2) for w in waves]
        print(json.dumps(out), flush=True)
        return 0
    finally:
        if frontend is not None and frontend.poll() is None:
            try:
                frontend.stdin.write("exit\n")
                frontend.stdin.flush()
                frontend.wait(120)
            except (OSError, sp.TimeoutExpired):
                frontend.kill()
                frontend.wait()
        shutil.rmtree(mof_dir, ignore_errors=True)


def run_api(args, ctx) -> int:
    """TeraSort through the C ABI: the same reduce-side work, entered the way the Hadoop plugins enter
    it (csrc/gpu/api_bench.cc). With N ranks every rank runs a MOFSupplier (TCP, its maps' outputs in
    its HBM) and `--reducers` reduce tasks that fetch their partition of every rank's maps as device
    descriptors (another rank's HBM is mapped over hipIpc, so the merge reads it over xGMI)."""
    import torch

    from uda_amd import native
    from uda_amd.models.terasort import RECORD_BYTES
    device = 0 if args.one_gpu else ctx.local_rank
    world, rank, R = ctx.world, ctx.rank, args.reducers
    # one provider per rank, all on one port at 127.0.0.<rank + 1> (providers of different hosts share the
    # port in Hadoop; -r of every reduce task)
    port = ctx.all_gather_object(_free_port() if rank == 0 else 0)[0] if world > 1 else 0
    hbm_bytes = 0
    if args.mof_dir:
        os.makedirs(args.mof_dir, exist_ok=True)
        _check_space(args.mof_dir, args.rows_per_gpu * RECORD_BYTES * (ctx.world if args.one_gpu else 1))
        per_rank = args.rows_per_gpu * RECORD_BYTES
        hbm_bytes = int(per_rank * 1.25) if args.provider_hbm_gb < 0 else int(args.provider_hbm_gb * 1e9)
    b = native().ApiTeraSortBench(dict(device=device, maps=args.maps_per_gpu, reducers=R,
                                       mof_dir=args.mof_dir, provider_hbm_bytes=hbm_bytes,
                                       workload=args.workload, skew=args.skew, codec=args.api_codec or "",
                                       records_per_map=max(1, args.rows_per_gpu // args.maps_per_gpu),
                                       round_bytes=args.round_mb << 20, rank=rank, world=world, port=port,
                                       transport="tcp" if world > 1 else "loopback",
                                       bind_addr=f"127.0.0.{rank + 1}" if world > 1 else "",
                                       host_mofs=args.api_host_mofs,
                                       # the measured best for 16 tasks whose map outputs are all in (6 slots)
                                       max_concurrent_merges=args.api_gpu_slots if args.api_gpu_slots >= 0 else
                                       (6 if args.api_host_mofs else -1),
                                       provider_workers=args.api_provider_workers,
                                       fetch=args.api_fetch or ("host" if args.api_host_mofs else "device")))
    t = time.perf_counter()
    b.setup()
    if world > 1:  # provider addresses and every task's expected record count (summed over the ranks' maps)
        b.set_peers([f"127.0.0.{p + 1}" for p in range(world)])
        parts = ctx.all_gather_object([int(x) for x in b.local_partition_records()])
        total = [sum(pr[g] for pr in parts) for g in range(world * R)]
        b.set_expected(total[rank * R:(rank + 1) * R])
    if rank == 0:
        print(f"# api setup {time.perf_counter() - t:.1f}s store={b.store_bytes/1e9:.1f}GB per rank, {world} rank(s)"
              f"{' on one GPU (rehearsal)' if args.one_gpu and world > 1 else ''}", file=sys.stderr, flush=True)
    first_step_ms = None
    for i in range(args.warmup):
        ctx.barrier()
        st = b.step(False)
        if first_step_ms is None:
            first_step_ms = st["wall_ms"]  # --mof-dir: includes the provider's first-touch file loads
        if args.verbose and rank == 0:
            print(f"# warmup {i}: {json.dumps(st)}", file=sys.stderr, flush=True)
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = [b.step(False) for _ in range(args.steps)]
    if first_step_ms is None:
        first_step_ms = stats[0]["wall_ms"]
    torch.cuda.synchronize()
    ctx.barrier()
    elapsed = ctx.max_float(time.perf_counter() - t0)
    validated = None
    if not args.no_validate:
        vst = b.step(True)
        validated = all(ctx.all_gather_object(vst["order_errors"] == 0))
        if args.verbose and rank == 0:
            print(f"# validated step: {json.dumps(vst)}", file=sys.stderr, flush=True)
    records = sum(ctx.all_gather_object(int(stats[0]["records"])))
    nbytes = sum(ctx.all_gather_object(int(stats[0]["bytes"])))  # delivered record bytes (EOF markers included)
    ms_per_step = elapsed * 1000.0 / max(1, args.steps)
    gbps = nbytes / (ms_per_step / 1000.0) / 1e9
    ctx.barrier()  # every rank's reduce tasks are done with the other ranks' providers
    if rank == 0:
        out = {
            "metric": "TeraSort shuffle+merge GB/s whole-node",
            "value": round(gbps, 3),
            "unit": "GB/s",
            "n_gpus": 1 if args.one_gpu else world,
            "ranks": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bytes",
            "data": ("synthetic secondary-sort map outputs generated in HBM: 22-62 byte Text keys sharing "
                     "5-50 byte prefixes, 0-120 byte values, "
                     f"{args.skew:.0%} of every map's records to reduce task 0" + (" of every rank" if world > 1 else ""))
                    if args.workload == "secondary" else
                    "synthetic TeraGen-shaped (10B key/90B value, 104B IFile records generated in HBM)",
            # device-wide, sampled (hipMemGetInfo): includes what no budget governs, the HIP runtime's own
            # HBM (context, code objects, scratch)
            "peak_hbm_gb": round(max(s["peak_hbm_bytes"] for s in stats) / 1e9, 2),
            # what the HBM ledger tracked at its peak during a timed step: reservations + pooled workspaces +
            # map outputs this process holds in HBM
            "hbm_ledger_peak_gb": round(max(s.get("hbm_ledger_peak_bytes", 0) for s in stats) / 1e9, 2),
            "hbm_budget_gb": round(stats[-1].get("hbm_budget_bytes", 0) / 1e9, 2),
            "hbm_budget_waits": int(stats[-1].get("hbm_budget_waits", 0)),
            # bytes allocated outside a reservation while the device was over its budget (0 = the budget held)
            "hbm_over_budget_bytes": int(stats[-1].get("hbm_over_budget_bytes", 0)),
            "max_task_ws_gb": round(max(s["max_task_ws_bytes"] for s in stats) / 1e9, 3),
            "max_task_rounds": int(max(s["max_task_rounds"] for s in stats)),
            "config": {
                "model": "secondary-sort" if args.workload == "secondary" else "terasort",
                "global_batch": records,
                "seq_len": RECORD_BYTES,
                "parallelism": f"dp{world}",
                "rows_per_gpu": args.rows_per_gpu,
                "maps_per_gpu": args.maps_per_gpu,
                "reducers_per_gpu": R,
                "shuffle": ("UdaBridge C ABI: uda_start/INIT/FETCH per reduce task, MOF files on disk found through "
                            "getPathUda, loaded once into the provider's HBM store and served as descriptors")
                           if args.mof_dir else
                           ("UdaBridge C ABI: uda_start/INIT/FETCH per reduce task, MOFs in host memory fetched "
                            f"as bytes (mapred.uda.gpu.fetch={args.api_fetch or 'host'}), merged on the GPU")
                           if args.api_host_mofs else
                           "UdaBridge C ABI: uda_start/INIT/FETCH per reduce task, HBM-resident MOFs "
                           "(descriptor fetch, merged in place" + ("; other ranks' MOFs mapped over hipIpc, "
                                                                    "fetch control over TCP)" if world > 1 else ")"),
                "delivery": "dataFromUda -> J2C consumer (KVBuf memcpy + VInt walk) per reduce task",
            },
            "reduce_wall_clock_s": round(ms_per_step / 1000.0, 3),
            "mof_files": bool(args.mof_dir),
            "codec": args.api_codec,
            "compressed_gb": round(b.compressed_bytes / 1e9, 2) if args.api_codec else None,
            "step_ms": [round(float(s["wall_ms"]), 1) for s in stats],  # this rank's timed steps
            "step_hbm_wait_ms": [[round(float(s.get("hbm_wait_ms_sum", 0)), 1), round(float(s.get("hbm_wait_ms_max", 0)), 1)]
                                 for s in stats],  # [sum over the tasks, slowest task]
            "step_task_ms_max": [round(float(s.get("task_total_ms_max", 0)), 1) for s in stats],
            "first_step_ms": round(first_step_ms, 1) if first_step_ms is not None else None,
            # --mof-dir: the first step includes every MOF file's load into the provider's HBM store (a
            # job loads each MOF once): this is the rate a job sees
            "first_step_gbps": round(nbytes / first_step_ms / 1e6, 3) if first_step_ms else None,
            "provider": json.loads(b.provider_stats()),
            "close_ms": round(sum(s["close_ms"] for s in stats) / len(stats), 2),
            "buffers_per_step": int(stats[0]["buffers"]),
            "task0_stats": json.loads(stats[0]["task0_stats"]) if stats[0]["task0_stats"] else None,
            "validated": validated,
            "reference_envelope_gbps_per_node": 5.0,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
