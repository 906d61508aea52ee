#!/usr/bin/env python3
"""Host-event trace of one NetMerger GPU task over host MOFs (2 GB secondary sort, loopback provider):
whole-partition early staging vs piecewise staging (mapred.uda.gpu.early.h2d.step) vs progressive
phases (mapred.uda.gpu.progressive.phases), taken apart from the UDA_HOST_TRACE events
(csrc/common/trace.cc):

  fetch_req    one transport request (issue -> completion callback)
  serve_copy   the provider worker's memcpy into the consumer's pinned span
  drain        one partition drained by a drain thread
  stage_wait   an H2D staging copy: queued -> issued to the SDMA engine
  stage_flush  the wait for every staged copy after the fetch
  fetch_phase / task  phase brackets

Prints one JSON line per variant (latency percentiles, memcpy GB/s, in-flight counts, 5 ms bins of
bytes landed), for docs/BENCHMARKS.md's fetch-slowdown analysis.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

TRACE = os.path.abspath(os.environ.setdefault("UDA_HOST_TRACE", "/tmp/uda_host_trace.csv"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def load(path):
    ev = []
    with open(path) as f:
        for line in f:
            k, tid, a, b, t0, t1 = line.rstrip("\n").split(",")
            ev.append((k, int(tid), int(a), int(b), int(t0), int(t1)))
    return ev


def pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def summarize(ev):
    task = [e for e in ev if e[0] == "task"][-1]
    t_start = task[4]
    fp = [e for e in ev if e[0] == "fetch_phase"][-1]
    out = {"task_ms": round((task[5] - task[4]) / 1e6, 1), "fetch_ms": round((fp[5] - fp[4]) / 1e6, 1)}
    for kind in ("fetch_req", "serve_copy", "drain", "index", "dm_h2d", "dm_merge", "rpq_deliver", "stage_wait", "lpq_flush", "lpq_merge", "lpq_d2h", "pinned_alloc",
                 "pinned_buf_alloc", "device_alloc", "device_free"):
        d = [(e[5] - e[4]) / 1e6 for e in ev if e[0] == kind]
        out[kind] = {"n": len(d), "p50_ms": pct(d, 0.5), "p90_ms": pct(d, 0.9), "max_ms": max(d) if d else None}
    sc = [e for e in ev if e[0] == "serve_copy"]
    if sc:
        gbps = [e[2] / max(e[5] - e[4], 1) for e in sc]  # bytes per ns = GB/s
        out["serve_copy"]["p50_gbps"] = round(pct(gbps, 0.5), 2)
        out["serve_copy"]["p10_gbps"] = round(pct(gbps, 0.1), 2)
        out["serve_copy"]["threads"] = len({e[1] for e in sc})
        # bytes landed per 5 ms bin, and mean memcpys in flight per bin
        end = max(e[5] for e in sc)
        t_start = min(t_start, min(e[4] for e in sc))  # copies may start before the task bracket opens
        nb = int((end - t_start) / 5e6) + 1
        landed = [0.0] * nb
        busy = [0.0] * nb
        for e in sc:
            landed[int((e[5] - t_start) / 5e6)] += e[2] / 1e6
            t = e[4]
            while t < e[5]:
                b = int((t - t_start) / 5e6)
                nxt = min(e[5], t_start + (b + 1) * 5e6)
                busy[b] += (nxt - t) / 5e6
                t = nxt
        out["landed_mb_per_5ms"] = [round(x) for x in landed]
        out["memcpys_in_flight_per_5ms"] = [round(x, 1) for x in busy]
    for kind in ("index", "dm_h2d", "dm_merge", "rpq_deliver", "lpq_flush", "lpq_merge", "lpq_d2h", "pinned_alloc", "pinned_buf_alloc", "device_alloc", "device_free"):  # spans vs task start
        sp = [e for e in ev if e[0] == kind]
        if sp:
            out[kind]["sum_ms"] = round(sum(e[5] - e[4] for e in sp) / 1e6, 1)
            out[kind]["spans_ms"] = [(round((e[4] - t_start) / 1e6, 1), round((e[5] - t_start) / 1e6, 1)) for e in sp]
    sf = [e for e in ev if e[0] == "stage_flush"]
    if sf:
        out["stage_flush_ms"] = round((sf[-1][5] - sf[-1][4]) / 1e6, 1)
        out["stage_copies"] = sf[-1][3]
    return out


def cpu_throttle():
    """(nr_throttled, throttled_usec) of this cgroup (v2 cpu.stat), or None: the GPU boxes run commands
    under a CPU quota, and a task whose threads exceed it inside a period stalls until the next one."""
    for path in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat", "/sys/fs/cgroup/cpu,cpuacct/cpu.stat"):
        try:
            kv = dict(line.split() for line in open(path))
        except OSError:
            continue
        usec = int(kv["throttled_usec"]) if "throttled_usec" in kv else int(kv.get("throttled_time", 0)) // 1000
        return int(kv.get("nr_throttled", 0)), usec
    return None


VMSTAT_KEYS = ("numa_hint_faults", "numa_hint_faults_local", "numa_pages_migrated", "pgmigrate_success",
               "compact_stall", "thp_fault_alloc", "thp_collapse_alloc", "pgmajfault", "pgfault", "tlb_remote_flush")


def vm_counters():
    """System-wide /proc/vmstat counters that can stall a process for tens of ms (NUMA hinting faults,
    compaction, THP) and this process's minor/major faults."""
    out = {}
    try:
        for line in open("/proc/vmstat"):
            k, v = line.split()
            if k in VMSTAT_KEYS:
                out[k] = int(v)
    except OSError:
        pass
    try:
        f = open("/proc/self/stat").read().rsplit(")", 1)[1].split()
        out["self_minflt"], out["self_majflt"] = int(f[7]), int(f[9])
    except (OSError, IndexError, ValueError):
        pass
    return out


class WchanSampler:
    """Every ~2 ms, the scheduler state and kernel wait channel of every thread of this process
    (/proc/self/task/*/stat, wchan): where threads sit while a task stalls. Samples of running
    threads and of the usual idle waits (futex, poll, sleep) are only counted."""
    IDLE = ("futex", "do_epoll_wait", "hrtimer_nanosleep", "do_sys_poll", "do_select", "pipe_read",
            "unix_stream_read", "inet_csk_accept", "0")

    def __init__(self):
        import threading
        self.samples = []
        self.futex = []  # (ms, thread name, futex word address)
        self.stop = threading.Event()
        self.t = threading.Thread(target=self.run, daemon=True)

    def run(self):
        t0 = time.perf_counter()
        while not self.stop.is_set():
            now = round((time.perf_counter() - t0) * 1e3, 1)
            for tid in os.listdir("/proc/self/task"):
                try:
                    st = open(f"/proc/self/task/{tid}/stat").read()
                    comm = st[st.index("(") + 1:st.rindex(")")]
                    state = st[st.rindex(")") + 2]
                    wchan = open(f"/proc/self/task/{tid}/wchan").read().strip()
                except (OSError, ValueError):
                    continue
                if wchan.startswith("futex"):  # which lock: the futex word's address (syscall arg 1)
                    try:
                        sc = open(f"/proc/self/task/{tid}/syscall").read().split()
                        if sc and sc[0] == "202":
                            self.futex.append((now, comm, int(sc[1], 16)))
                    except (OSError, ValueError, IndexError):
                        pass
                    continue
                if state == "R" or any(wchan.startswith(i) for i in self.IDLE):
                    continue
                self.samples.append((now, comm, state, wchan))
            time.sleep(0.002)

    def summary(self):
        from collections import Counter
        c = Counter((w, st) for _, _, st, w in self.samples)
        maps = []
        try:
            for line in open("/proc/self/maps"):
                f = line.split()
                lo, hi = (int(x, 16) for x in f[0].split("-"))
                maps.append((lo, hi, f[5] if len(f) > 5 else "[anon]"))
        except OSError:
            pass
        def where(a):
            for lo, hi, name in maps:
                if lo <= a < hi:
                    return f"{name}+0x{a - lo:x}"
            return "?"
        # futex words waited on by several threads in the same sample: contended locks
        per_t = {}
        for t, comm, a in self.futex:
            per_t.setdefault((t, a), set()).add(comm)
        contended = Counter()
        names = {}
        for (t, a), comms in per_t.items():
            if len(comms) >= 3:
                contended[a] += 1
                names.setdefault(a, set()).update(comms)
        return {"busy_waits": [[w, st, n] for (w, st), n in c.most_common(12)],
                "contended_futex": [[hex(a), where(a), n, sorted(names[a])[:6]] for a, n in contended.most_common(6)],
                "first": self.samples[:20]}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=2.0)
    ap.add_argument("--maps", type=int, default=64)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--wchan", action="store_true", help="sample every thread's kernel wait channel")
    ap.add_argument("--variants", default="whole,step8m,step32m",
                    help="comma list of whole, step8m, step32m, prog2, prog4, prog8, prog16")
    args = ap.parse_args()
    for f in ("/proc/sys/kernel/numa_balancing", "/sys/kernel/mm/transparent_hugepage/enabled",
              "/sys/kernel/mm/transparent_hugepage/defrag"):
        try:
            print(f"# {f}: {open(f).read().strip()}", file=sys.stderr, flush=True)
        except OSError:
            pass
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
        prov.add_mof_memory("job_tr", f"attempt_tr_m_{m:06d}_0", data, index)
    del runs
    named = {"whole": {}, "step8m": {"mapred.uda.gpu.early.h2d.step": 8 << 20},
             "step32m": {"mapred.uda.gpu.early.h2d.step": 32 << 20}}
    for ph in (2, 4, 8, 16):
        named[f"prog{ph}"] = {"mapred.uda.gpu.progressive.phases": ph}
    named["whole"] = {"mapred.uda.gpu.progressive.phases": 0}
    named["hybrid"] = {"mapred.uda.gpu.merge.bytes": max(1 << 20, total // 6), "mapred.uda.gpu.spill": "host"}
    named["hybrid_lpq"] = {**named["hybrid"], "mapred.uda.gpu.hybrid.direct": 0}
    named["whole_nopw"] = {**named["whole"], "mapred.uda.gpu.prewarm": 0}
    named["prog4_nopw"] = {"mapred.uda.gpu.progressive.phases": 4, "mapred.uda.gpu.prewarm": 0}
    variants = [("warmup", {})] + [(f"{name}_{i}", named[name]) for i in range(args.repeat)
                                   for name in args.variants.split(",")]
    for i, (name, extra) in enumerate(variants):
        if os.path.exists(TRACE):
            os.unlink(TRACE)
        conf = {"mapred.uda.merge.backend": "gpu", **extra}
        c = UdaConsumer(args.maps, "job_tr", f"attempt_tr_r_{i:06d}_0", TEXT, conf=conf, keep_records=False)
        thr0 = cpu_throttle()
        vm0 = vm_counters()
        ws = WchanSampler() if args.wchan else None
        if ws:
            ws.t.start()
        t0 = time.perf_counter()
        for m in range(args.maps):
            c.fetch("localhost", "job_tr", f"attempt_tr_m_{m:06d}_0", 0)
        c.wait(3600)
        wall = time.perf_counter() - t0
        st = c.close()
        if ws:
            ws.stop.set()
            ws.t.join()
        assert st["bytes_delivered"] - 2 == total, (st["bytes_delivered"], total)
        res = {"variant": name, "gbps": round(total / wall / 1e9, 2), "wall_ms": round(wall * 1e3, 1),
               "lpqs": st.get("lpqs"), "spill_bytes": st.get("spill_bytes"),
               "phases_ms": {k: round(st["gpu_" + k + "_ms"], 1) for k in ("h2d", "device", "d2h_wait", "sink")},
               "fetch_ms_stat": round(st["fetch_ms"], 1), "merge_ms_stat": round(st["merge_ms"], 1),
               "progressive_rounds": st.get("rpq_rounds"), "hybrid_direct": st.get("hybrid_direct"),
               "prewarm_ms": st.get("gpu_prewarm_ms"), "prewarm_wait_ms": st.get("gpu_prewarm_wait_ms")}
        thr1 = cpu_throttle()
        vm1 = vm_counters()
        if ws:
            res["wchan"] = ws.summary()
        res["vm_deltas"] = {k: vm1[k] - vm0[k] for k in vm1 if k in vm0 and vm1[k] != vm0[k]}
        if thr0 and thr1:
            res["cpu_throttled"] = {"periods": thr1[0] - thr0[0], "ms": round((thr1[1] - thr0[1]) / 1e3, 1)}
        if name != "warmup" and os.path.exists(TRACE):
            res.update(summarize(load(TRACE)))
        print(json.dumps(res), flush=True)
    prov.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
