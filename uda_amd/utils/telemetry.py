"""Per-node resource telemetry sampled during a run (the reference's dstat collection).

Reference: scripts/regression/mr-dstatExcel.sh:89-201 runs `dstat` on every node during each
test and turns the CSVs into per-node CPU/disk/network sheets (SURVEY.md §5 "Tracing /
profiling"). Here a background thread samples the host (psutil: CPU %, memory, disk and network
bytes/s) and every visible AMD GPU through sysfs (busy %, VRAM used) at a fixed interval and writes
one CSV row per sample; `summary()` reduces it to mean/peak figures for reports.

    with Telemetry("out/sample0.dstat.csv", interval=1.0) as t:
        run_job(...)
    print(t.summary())
"""
from __future__ import annotations

import csv
import glob
import os
import threading
import time

try:
    import psutil
except ImportError:  # pragma: no cover - psutil ships in this image; keep the sampler optional
    psutil = None

FIELDS = ["t_s", "cpu_pct", "mem_used_gb", "disk_read_mbs", "disk_write_mbs", "net_recv_mbs", "net_sent_mbs"]


def _gpu_nodes() -> list[str]:
    """sysfs device dirs of AMD GPUs (those exposing gpu_busy_percent)."""
    return sorted(os.path.dirname(p) for p in glob.glob("/sys/class/drm/card*/device/gpu_busy_percent"))


def _read_int(path: str) -> int | None:
    try:
        with open(path) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return None


class Telemetry:
    def __init__(self, path: str | None, interval: float = 1.0):
        self.path = path
        self.interval = interval
        self.rows: list[dict] = []
        self.gpus = _gpu_nodes()
        self._stop = threading.Event()
        self._thr: threading.Thread | None = None

    def fields(self) -> list[str]:
        f = list(FIELDS)
        for i in range(len(self.gpus)):
            f += [f"gpu{i}_busy_pct", f"gpu{i}_vram_gb"]
        return f

    def _sample(self, t0: float, prev: dict) -> dict:
        now = time.perf_counter()
        dt = max(1e-6, now - prev.get("now", t0))
        row = {"t_s": round(now - t0, 3)}
        if psutil is not None:
            row["cpu_pct"] = psutil.cpu_percent(interval=None)
            row["mem_used_gb"] = round(psutil.virtual_memory().used / 1e9, 3)
            d = psutil.disk_io_counters()
            n = psutil.net_io_counters()
            if d is not None and "disk" in prev:
                row["disk_read_mbs"] = round((d.read_bytes - prev["disk"].read_bytes) / dt / 1e6, 2)
                row["disk_write_mbs"] = round((d.write_bytes - prev["disk"].write_bytes) / dt / 1e6, 2)
            if n is not None and "net" in prev:
                row["net_recv_mbs"] = round((n.bytes_recv - prev["net"].bytes_recv) / dt / 1e6, 2)
                row["net_sent_mbs"] = round((n.bytes_sent - prev["net"].bytes_sent) / dt / 1e6, 2)
            prev["disk"], prev["net"] = d, n
        for i, g in enumerate(self.gpus):
            row[f"gpu{i}_busy_pct"] = _read_int(os.path.join(g, "gpu_busy_percent"))
            v = _read_int(os.path.join(g, "mem_info_vram_used"))
            row[f"gpu{i}_vram_gb"] = round(v / 1e9, 3) if v is not None else None
        prev["now"] = now
        return row

    def _run(self) -> None:
        t0 = time.perf_counter()
        prev: dict = {}
        if psutil is not None:
            psutil.cpu_percent(interval=None)  # prime the CPU counter
        self._sample(t0, prev)
        while not self._stop.wait(self.interval):
            self.rows.append(self._sample(t0, prev))
        self.rows.append(self._sample(t0, prev))

    def start(self) -> "Telemetry":
        self._thr = threading.Thread(target=self._run, name="uda-telemetry", daemon=True)
        self._thr.start()
        return self

    def stop(self) -> None:
        if self._thr is None:
            return
        self._stop.set()
        self._thr.join()
        self._thr = None
        if self.path:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
            with open(self.path, "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=self.fields(), extrasaction="ignore")
                w.writeheader()
                w.writerows(self.rows)

    def __enter__(self) -> "Telemetry":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()

    def summary(self) -> dict:
        """mean and peak of every numeric column over the samples."""
        out = {"samples": len(self.rows)}
        for k in self.fields()[1:]:
            xs = [r[k] for r in self.rows if isinstance(r.get(k), (int, float))]
            if xs:
                out[k] = {"mean": round(sum(xs) / len(xs), 2), "peak": max(xs)}
        return out
