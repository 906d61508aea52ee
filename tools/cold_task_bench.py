#!/usr/bin/env python3
"""Cold reduce task: one NetMerger GPU task in a fresh process, the way Hadoop runs every reduce task
in its own JVM. INIT comes first; after `--gap` seconds (the reduce slow-start window, maps still
running) the 64 FETCHes arrive. Measured from the first FETCH to the EOF: the task's own time, with
the INIT-time GPU prewarm (mapred.uda.gpu.prewarm, default) and without it.

Each trial is a child process (`--child`), so HIP, the pools and the code objects start cold. Prints
one JSON line per trial."""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(args) -> int:
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
        prov.add_mof_memory("job_cold", f"attempt_cold_m_{m:06d}_0", data, index)
    del runs
    conf = {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.prewarm": args.prewarm}
    c = UdaConsumer(args.maps, "job_cold", "attempt_cold_r_000000_0", TEXT, conf=conf, keep_records=False)
    time.sleep(args.gap)
    t0 = time.perf_counter()
    for m in range(args.maps):
        c.fetch("localhost", "job_cold", f"attempt_cold_m_{m:06d}_0", 0)
    c.wait(600)
    wall = time.perf_counter() - t0
    st = c.close()
    prov.close()
    assert st["bytes_delivered"] - 2 == total, (st["bytes_delivered"], total)
    trace = {}
    tr = os.environ.get("UDA_HOST_TRACE")
    if tr and os.path.exists(tr):  # host-event breakdown of the task (tools/netmerger_trace.py)
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import netmerger_trace
        trace = netmerger_trace.summarize(netmerger_trace.load(tr))
        os.unlink(tr)
    print(json.dumps({"prewarm": args.prewarm, "gap_s": args.gap, "gb": round(total / 1e9, 3),
                      "gbps": round(total / wall / 1e9, 2), "wall_ms": round(wall * 1e3, 1),
                      "fetch_ms": round(st["fetch_ms"], 1), "merge_ms": round(st["merge_ms"], 1),
                      "prewarm_ms": round(st.get("gpu_prewarm_ms", -1), 1),
                      "prewarm_wait_ms": round(st.get("gpu_prewarm_wait_ms", 0), 1),
                      "merge_path": st.get("merge_path"), **({"trace": trace} if trace else {})}), flush=True)
    return 0


def node(args) -> int:
    """The node shape of a cold reduce task: this process is the node's MOFSupplier (host MOFs, TCP, long
    lived and warm, as the NodeManager aux service is), and every trial starts a fresh uda_reduce_task
    process (its ReduceTask JVM): INIT, the slow-start gap, then the FETCHes; the task reports FETCH ->
    EOF. With the merge service the task's NetMerger runs in this process (warm GPU context and pools)
    and the task process only reads the merged buffers in place; without it the task merges in its own
    process (prewarm during the gap)."""
    import socket
    import time
    from uda_amd import native
    from uda_amd.bridge import FETCH, INIT, UdaProvider
    from uda_amd.utils.datagen import TEXT
    from uda_amd.utils.mof import encode_partitions
    n = native()
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "uda_amd", "bin", "uda_reduce_task")
    rows = int(args.gb * 1e9 / 100 / args.maps)
    runs = n.generate_runs("secondary", args.maps, 1, rows, 9)
    mofs = []
    for m, parts in enumerate(runs):
        data, index = encode_partitions(parts)
        mofs.append((f"attempt_cold_m_{m:06d}_0", data, index, n.ifile_checksum(parts[0])[0]))
    del runs
    total = sum(len(d) - 2 for _, d, _, _ in mofs)
    expect = sum(c for _, _, _, c in mofs)
    child_env = {k: v for k, v in os.environ.items() if k != "UDA_HOST_TRACE"}  # the trace is this process's
    for svc in ((1,) if args.service_only else (1, 0)):
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        path = f"/tmp/uda-cold-{os.getpid()}.sock"
        conf = {"mapred.uda.provider.bind.address": "127.0.0.1"}
        if svc:
            conf["mapred.uda.gpu.merge.service"] = path
        prov = UdaProvider(transport="tcp", data_port=port, conf=conf)
        try:
            for mid, data, index, _ in mofs:
                prov.add_mof_memory("job_cold", mid, data, index)
            for t in range(args.repeat + 1):  # trial 0 warms the service's pools (a node's first task)
                argv = [exe, "-D", "mapred.uda.transport=tcp", "-D", f"mapred.uda.merge.backend={args.backend}",
                        "-D", f"mapred.uda.gpu.prewarm={args.prewarm}", "--expect", str(expect)]
                if t == args.repeat:  # the last trial also checks the key order of every record (slower walk)
                    argv.append("--check-order")
                if svc:
                    argv += ["-D", f"mapred.uda.gpu.merge.service={path}"]
                for kv in args.conf:
                    argv += ["-D", kv]
                argv += ["--", "-w", "256", "-r", str(port), "-a", "1", "-m", "1", "-g", "/tmp", "-s", "1024"]
                init = n.form_cmd(INIT, [str(args.maps), "job_cold", "attempt_cold_r_000000_0", "0", str(1 << 20),
                                         str(16 << 10), TEXT, "null", str(256 << 10), "0", "0"])
                p = subprocess.Popen(argv, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=child_env)
                p.stdin.write(init + "\n")
                p.stdin.flush()
                time.sleep(args.gap)
                p.stdin.write("\n".join(n.form_cmd(FETCH, ["127.0.0.1", "job_cold", mid, "0"]) for mid, _, _, _ in mofs) + "\n")
                p.stdin.close()
                out = p.stdout.read()
                p.wait(timeout=300)
                res = json.loads(out.strip().splitlines()[-1])
                if p.returncode != 0 or res.get("error"):
                    print(json.dumps({"error": res.get("error"), "rc": p.returncode}), flush=True)
                    return 1
                st = res["task"]
                print(json.dumps({"mode": "node", "merge_service": bool(svc), "trial": t, "gap_s": args.gap,
                                  "order_checked": t == args.repeat,
                                  "gb": round(total / 1e9, 3), "gbps": round(total / res["fetch_to_eof_ms"] / 1e6, 2),
                                  "fetch_to_eof_ms": res["fetch_to_eof_ms"], "exec_to_end_ms": res["exec_to_end_ms"],
                                  "fetch_ms": round(st.get("fetch_ms", -1), 1), "merge_ms": round(st.get("merge_ms", -1), 1),
                                  "prewarm_wait_ms": round(st.get("gpu_prewarm_wait_ms", 0), 1),
                                  "fetch_to_first_data_ms": res["fetch_to_first_data_ms"],
                                  **{k: round(st.get(k, -1), 1) for k in ("gpu_h2d_ms", "gpu_device_ms", "gpu_d2h_wait_ms",
                                                                           "gpu_sink_ms")},
                                  "merge_path": st.get("merge_path"), "j2c": res.get("j2c")}), flush=True)
        finally:
            prov.close()
    return 0


def files(args) -> int:
    """The documented deployment for one cold task: TeraSort map outputs written as Hadoop-layout MOF
    files, the provider front end (uda_mof_supplier mode=frontend, library defaults: node daemon with
    the HBM store and the merge service), and every trial a fresh uda_reduce_task process with no
    mapred.uda.* key. Trial 0 reads the files from disk into the store (a job's first reducer touching
    them); later trials are cold task processes over a warm store, as every later reducer of the job."""
    import shutil
    import socket
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    bindir = os.path.join(root, "uda_amd", "bin")
    exe, sup = os.path.join(bindir, "uda_reduce_task"), os.path.join(bindir, "uda_mof_supplier")
    mof_dir = tempfile.mkdtemp(prefix="uda-cold-files-", dir=args.mof_dir)
    fe = None
    try:
        recs = int(args.gb * 1e9 / 104 / args.maps)
        g = subprocess.run([sup, "mode=mapgen", f"mof_dir={mof_dir}", "device=0", f"maps={args.maps}", "reducers=1",
                            f"records_per_map={recs}", "workload=terasort"], stdout=subprocess.PIPE, text=True,
                           timeout=600)
        job = json.loads(g.stdout.strip().splitlines()[-1])
        cmds, expect = job["commands"][0], job["expected"][0]
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        fe = subprocess.Popen([sup, "mode=frontend", f"mof_dir={mof_dir}", f"port={port}"], stdin=subprocess.PIPE,
                              stdout=subprocess.PIPE, text=True)
        json.loads(fe.stdout.readline())
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 120:  # the node daemon and its prewarm, as a job finds them
            fe.stdin.write("stats\n")
            fe.stdin.flush()
            hs = json.loads(fe.stdout.readline()).get("hbm_store", {})
            if hs.get("daemon", {}).get("ready") and hs.get("prewarm", {}).get("done", True):
                break
            time.sleep(0.2)
        start = ["-w", "256", "-r", str(port), "-a", "1", "-m", "1", "-g", "/tmp", "-s", "1024"]
        for t in range(args.repeat + 1):
            argv = [exe, "--expect", str(expect)] + (["--check-order"] if t == args.repeat else [])
            for kv in args.conf:
                argv += ["-D", kv]
            p = subprocess.Popen(argv + ["--"] + start, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
            p.stdin.write(cmds[0] + "\n")
            p.stdin.flush()
            time.sleep(args.gap)
            p.stdin.write("\n".join(cmds[1:]) + "\n")
            p.stdin.close()
            out = p.stdout.read()
            p.wait(timeout=300)
            res = json.loads(out.strip().splitlines()[-1])
            if p.returncode != 0 or res.get("error"):
                print(json.dumps({"error": res.get("error"), "rc": p.returncode}), flush=True)
                return 1
            st = res["task"]
            print(json.dumps({"mode": "files", "trial": t, "store": "cold (files read)" if t == 0 else "warm",
                              "order_checked": t == args.repeat, "gb": round(res["bytes"] / 1e9, 3),
                              "gbps": round(res["bytes"] / res["fetch_to_eof_ms"] / 1e6, 2),
                              "fetch_to_eof_ms": res["fetch_to_eof_ms"], "fetch_to_first_data_ms": res["fetch_to_first_data_ms"],
                              "fetch_ms": round(st.get("fetch_ms", -1), 1), "merge_ms": round(st.get("merge_ms", -1), 1),
                              "gpu_sink_ms": round(st.get("gpu_sink_ms", -1), 1), "merge_service": st.get("merge_service"),
                              "merge_path": st.get("merge_path"), "j2c": res.get("j2c")}), flush=True)
        return 0
    finally:
        if fe is not None and fe.poll() is None:
            fe.stdin.write("exit\n")
            fe.stdin.flush()
            fe.wait(120)
        shutil.rmtree(mof_dir, ignore_errors=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=2.0)
    ap.add_argument("--maps", type=int, default=64)
    ap.add_argument("--gap", type=float, default=1.0)
    ap.add_argument("--prewarm", type=int, default=1)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--backend", default="gpu", help="--node: mapred.uda.merge.backend of the tasks")
    ap.add_argument("--service-only", action="store_true", help="--node: only the merge-service trials")
    ap.add_argument("--conf", action="append", default=[], help="--node/--files: extra -D key=value of every task")
    ap.add_argument("--files", action="store_true",
                    help="MOF files -> provider front end with library defaults (node daemon, HBM store, merge "
                         "service) -> each trial a fresh uda_reduce_task with no mapred.uda.* key")
    ap.add_argument("--mof-dir", default="/tmp", help="--files: where the MOF files are written")
    ap.add_argument("--node", action="store_true",
                    help="provider (and merge service) in this process, each task a fresh uda_reduce_task process")
    args = ap.parse_args()
    if args.child:
        return child(args)
    if args.files:
        return files(args)
    if args.node:
        return node(args)
    for _ in range(args.repeat):
        for pw in (1, 0):
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--gb", str(args.gb),
                                "--maps", str(args.maps), "--gap", str(args.gap), "--prewarm", str(pw)],
                               timeout=300)
            if r.returncode != 0:
                return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
