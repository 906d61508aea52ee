"""MapReduce shuffle jobs through the plugin path: MOFSupplier -> fetch -> NetMerger -> dataFromUda.

The workload families of the reference's regression matrix (scripts/regression/sortcountRunner.sh:
terasort, sort, wordcount) as runnable jobs on this framework. A job generates
synthetic map outputs of its program's shape, serves them from a provider (in process over the
loopback transport, or from a separate process over TCP), runs one NetMerger per reducer with the
chosen merge backend, and validates every reducer's delivered stream natively (teravalidate:
framing, key order, record count, checksum against the map outputs).

    from uda_amd.models.jobs import ShuffleJobSpec, run_job
    res = run_job(ShuffleJobSpec(program="secondary", gb=0.2, backend="gpu"))
    res["gbps"], res["valid"]

The TeraSort flagship with all data resident in HBM and an RCCL all-to-all is
uda_amd/models/terasort.py (bench.py); this module is the host-plugin path the reference ships.
"""
from __future__ import annotations

import dataclasses
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

from .._native import native
from ..bridge import UdaConsumer, UdaProvider
from ..utils.mof import encode_partitions, write_mof

TEXT = "org.apache.hadoop.io.Text"
# native generator kind and approximate serialized bytes per record (csrc/engine/datagen.cc)
PROGRAMS = {
    "terasort": ("terasort", 104, TEXT),
    "wordcount": ("wordcount", 17, TEXT),
    "secondary": ("secondary", 100, TEXT),
}


@dataclasses.dataclass
class ShuffleJobSpec:
    program: str = "wordcount"      # terasort | wordcount | secondary
    maps: int = 16
    reducers: int = 4
    gb: float = 0.1                 # total map-output bytes (uncompressed)
    codec: str | None = None        # None | snappy | lzo
    backend: str = "cpu"            # cpu (heap merge, the reference algorithm) | gpu (HIP merge)
    approach: int = 1               # 1 online | 2 hybrid (LPQ spill + RPQ)
    transport: str = "loopback"     # loopback | tcp (provider in another process)
    seed: int = 7
    gpu_merge_bytes: int = 0        # >0: device budget per merge (forces the GPU hybrid when smaller)
    kv_buf_size: int = 1 << 20
    max_buf_kb: int = 1024
    log_level: int = 4              # native log threshold: 4 = info (the health lines are info)

    @classmethod
    def from_dict(cls, d: dict) -> "ShuffleJobSpec":
        names = {f.name: f for f in dataclasses.fields(cls)}
        out = {}
        for k, v in d.items():
            if k not in names or v in ("", None):
                continue
            t = names[k].type
            if k == "codec":
                out[k] = None if str(v).lower() in ("none", "null", "") else str(v)
            elif "int" in str(t):
                out[k] = int(v)
            elif "float" in str(t):
                out[k] = float(v)
            else:
                out[k] = str(v)
        return cls(**out)


_TCP_PROVIDER = r"""
import json, sys
sys.path.insert(0, sys.argv[3])
from uda_amd.bridge import UdaProvider
p = UdaProvider(transport="tcp", data_port=int(sys.argv[1]), log_level=int(sys.argv[4]))
for job, mid, path in json.loads(sys.argv[2]):
    p.add_mof_file(job, mid, path)
print("READY", flush=True)
sys.stdin.read()
p.close()
for s, m in p.logs:
    print("LOG", s, m, flush=True)
"""


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_job(spec: ShuffleJobSpec, workdir: str | None = None, timeout: float = 3600.0) -> dict:
    """Run one shuffle job; returns timings, per-reducer stats, validation and the native logs."""
    if spec.program not in PROGRAMS:
        raise ValueError(f"unknown program {spec.program!r}")
    kind, row_bytes, key_class = PROGRAMS[spec.program]
    n = native()
    rows = max(1, int(spec.gb * 1e9 / row_bytes / spec.maps))
    t0 = time.perf_counter()
    runs = n.generate_runs(kind, spec.maps, spec.reducers, rows, spec.seed)
    gen_s = time.perf_counter() - t0
    job = f"job_{spec.program}_{spec.seed}"
    mids = [f"attempt_{job}_m_{m:06d}_0" for m in range(spec.maps)]
    # expected per-reducer records/checksum from the (uncompressed) map outputs
    want = [[0, 0, 0] for _ in range(spec.reducers)]
    for parts in runs:
        for r, part in enumerate(parts):
            recs, nbytes, ck = n.ifile_checksum(part)
            want[r][0] += recs
            want[r][1] += nbytes
            want[r][2] = (want[r][2] + ck) % (1 << 64)
    total = sum(w[1] for w in want)

    tmp = None
    provider = proc = None
    logs: list[str] = []
    conf = {"mapred.uda.merge.backend": spec.backend}
    if spec.gpu_merge_bytes > 0:
        conf["mapred.uda.gpu.merge.bytes"] = spec.gpu_merge_bytes
    local_dirs: tuple[str, ...] = ()
    if spec.approach == 2 or spec.gpu_merge_bytes > 0 or spec.transport == "tcp":
        tmp = tempfile.mkdtemp(prefix="uda_job_", dir=workdir)
        local_dirs = (tmp,)
    try:
        if spec.transport == "tcp":
            mofs = []
            for mid, parts in zip(mids, runs):
                path, _ = write_mof(tmp, mid, parts, codec=spec.codec)
                mofs.append((job, mid, path))
            port = _free_port()
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            proc = subprocess.Popen([sys.executable, "-c", _TCP_PROVIDER, str(port), json.dumps(mofs), root,
                                     str(spec.log_level)],
                                    stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
            if proc.stdout.readline().strip() != "READY":
                raise RuntimeError("TCP provider did not start")
        else:
            port = 9011
            provider = UdaProvider(log_level=spec.log_level)
            for mid, parts in zip(mids, runs):
                data, index = encode_partitions(parts, codec=spec.codec)
                provider.add_mof_memory(job, mid, data, index)
        del runs
        consumers = [UdaConsumer(spec.maps, job, f"attempt_{job}_r_{r:06d}_0", key_class, codec=spec.codec,
                                 conf=conf, approach=spec.approach, local_dirs=local_dirs, transport=spec.transport,
                                 data_port=port, max_buf_kb=spec.max_buf_kb, kv_buf_size=spec.kv_buf_size,
                                 keep_records=False, validate=True, log_level=spec.log_level)
                     for r in range(spec.reducers)]
        t0 = time.perf_counter()
        for r, c in enumerate(consumers):
            for mid in mids:
                c.fetch("127.0.0.1" if spec.transport == "tcp" else "localhost", job, mid, r)
        failures = []
        for r, c in enumerate(consumers):
            try:
                c.wait(timeout)
            except Exception as e:  # noqa: BLE001  (fallback / timeout are results, not crashes)
                failures.append(f"reducer {r}: {e}")
        wall = time.perf_counter() - t0
        stats = [c.close() for c in consumers]
        for c in consumers:
            logs += [f"[consumer {s}] {m}" for s, m in c.logs]
    finally:
        if provider is not None:
            provider.close()
            logs += [f"[provider {s}] {m}" for s, m in provider.logs]
        if proc is not None:
            proc.stdin.close()
            out = proc.stdout.read()
            proc.wait(timeout=60)
            logs += ["[provider " + ln[4:].split(" ", 1)[0] + "] " + ln[4:].split(" ", 1)[-1]
                     for ln in out.splitlines() if ln.startswith("LOG ")]
        if tmp is not None:
            import shutil
            shutil.rmtree(tmp, ignore_errors=True)

    per = []
    valid = not failures
    for r, c in enumerate(consumers):
        v = c.validator
        ok = (v.eof and v.order_errors == 0 and v.framing_errors == 0 and v.records == want[r][0]
              and v.checksum == want[r][2] and v.bytes == want[r][1])
        valid &= ok
        per.append({"reducer": r, "records": v.records, "bytes": v.bytes, "buffers": v.buffers,
                    "order_errors": v.order_errors, "framing_errors": v.framing_errors,
                    "checksum_ok": v.checksum == want[r][2], "valid": ok, "failure_calls": c.failure_calls,
                    "stats": stats[r]})
    return {"spec": dataclasses.asdict(spec), "bytes": total, "wall_s": wall, "gbps": total / wall / 1e9,
            "gen_s": gen_s, "valid": valid, "failures": failures, "reducers": per, "logs": logs}
