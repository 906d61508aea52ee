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


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=2.0)
    ap.add_argument("--maps", type=int, default=64)
    ap.add_argument("--gap", type=float, default=1.0)
    ap.add_argument("--prewarm", type=int, default=1)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        return child(args)
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
