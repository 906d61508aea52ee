"""Host side of the UdaBridge API: a Python stand-in for the Java plugin classes.

The reference's Java layer (plugins/shared/com/mellanox/hadoop/mapred/*) drives libuda.so through
four natives and six callbacks. The same contract is exercised here through the C ABI:

  UdaConsumer  ~ UdaPluginRT + UdaShuffleConsumerPluginShared (UdaPlugin.java:146-556): builds the
               CLI args, sends INIT and FETCH commands, receives merged buffers in `dataFromUda`
               (parsed by a J2CQueue-equivalent reader), tracks fetch progress via
               `fetchOverMessage`, and on `failureInUda` marks the task for fallback.
  UdaProvider  ~ UdaShuffleProviderPluginShared + UdaPluginTT/SH (getPathIndex): starts the
               MOFSupplier and resolves (job, map, reduce) to MOF index records.
"""
from __future__ import annotations

import os
import threading
import time

from ._native import native
from .utils.ifile import J2CQueueReader
from .utils.mof import CODEC_CLASSES, read_index

EXIT, NEW_MAP, FINAL, RESULT, FETCH, FETCH_OVER, JOB_OVER, INIT, MORE, RT_LAUNCHED = range(10)
PROGRESS_REPORT_LIMIT = 20


class UdaFallback(RuntimeError):
    """Raised where the Java plugin would fall back to the vanilla Hadoop shuffle."""


class _Conf:
    def __init__(self, conf: dict | None):
        self.conf = dict(conf or {})

    def __call__(self, key: str, default: str) -> str:
        v = self.conf.get(key)
        return default if v is None else str(v)


class UdaProvider:
    """MOFSupplier host (TaskTracker / NodeManager aux-service side)."""

    def __init__(self, conf: dict | None = None, transport: str = "loopback", data_port: int = 9011,
                 log_level: int = 3, loopback_host: str = "*"):
        self.mofs: dict[tuple[str, str], tuple[str, list]] = {}
        self.logs: list[tuple[int, str]] = []
        conf = dict(conf or {})
        conf.setdefault("mapred.uda.transport", transport)
        conf.setdefault("mapred.uda.loopback.host", loopback_host)
        self._conf = _Conf(conf)
        args = ["-w", str(conf.get("mapred.rdma.wqe.per.conn", 256)), "-r", str(data_port), "-m", "1",
                "-g", "/tmp", "-s", str(conf.get("mapred.rdma.buf.size", 1024))]
        self.bridge = native().Bridge(False, args, log_level, get_path=self._get_path, get_conf=self._conf,
                                      log=lambda m, s: self.logs.append((s, m)))

    def add_mof_file(self, job_id: str, map_id: str, file_out: str) -> None:
        """Register an on-disk MOF; its index is read from file.out.index (getPathIndex)."""
        self.mofs[(job_id, map_id)] = (file_out, read_index(file_out + ".index"))

    def add_mof_memory(self, job_id: str, map_id: str, data: bytes, index: list) -> None:
        flat = [v for rec in index for v in rec]
        if self.bridge.register_mof(job_id, map_id, data, flat) != 0:
            raise RuntimeError("register_mof failed")

    def add_mof_device(self, job_id: str, map_id: str, data: bytes, index: list, device: int = 0):
        """Register an HBM-resident MOF: `data` is copied to device `device` (a torch tensor kept
        alive by the provider) and reducers on the GPU backend merge its partitions in place."""
        import torch
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(f"cuda:{device}")
        self._keep = getattr(self, "_keep", [])
        self._keep.append(t)
        self.add_mof_device_ptr(job_id, map_id, t.data_ptr(), t.numel(), index, device)
        return t

    def add_mof_device_ptr(self, job_id: str, map_id: str, ptr: int, nbytes: int, index: list, device: int = 0):
        flat = [v for rec in index for v in rec]
        if self.bridge.register_mof_device(job_id, map_id, ptr, nbytes, flat, device) != 0:
            raise RuntimeError("register_mof_device failed")

    def _get_path(self, job_id: str, map_id: str, reduce_id: int):
        ent = self.mofs.get((job_id, map_id))
        if ent is None or reduce_id >= len(ent[1]):
            return None
        start, raw, part = ent[1][reduce_id]
        return (start, raw, part, ent[0])

    def stats(self) -> str:
        return self.bridge.stats()

    def close(self) -> None:
        self.bridge.do_command(native().form_cmd(EXIT, []))


class UdaConsumer:
    """NetMerger host for one reduce task."""

    def __init__(self, num_maps: int, job_id: str, reduce_task_id: str, key_class: str,
                 codec: str | None = None, conf: dict | None = None, approach: int = 1,
                 local_dirs: tuple[str, ...] = (), transport: str = "loopback", data_port: int = 9011,
                 max_buf_kb: int = 1024, min_buf_kb: int = 16, shuffle_mem: int = 0, lpq_size: int = 0,
                 comp_block_size: int = 256 * 1024, kv_buf_size: int = 1 << 20, log_level: int = 3,
                 keep_records: bool = True, validate: bool = False):
        self.num_maps = num_maps
        self.reader = J2CQueueReader(max_len=kv_buf_size) if keep_records else None
        # teravalidate in native code (framing, order, checksum) without keeping the records
        self.validator = native().StreamValidator(key_class) if validate else None
        self.bytes = 0
        self.buffers = 0
        self.maps_reported = 0
        self.fetch_over_calls = 0
        self.failure: str | None = None
        self.failure_calls = 0
        self.logs: list[tuple[int, str]] = []
        self._done = threading.Event()
        conf = dict(conf or {})
        conf.setdefault("mapred.uda.transport", transport)
        conf.setdefault("mapred.uda.kv.buf.size", kv_buf_size)
        self._conf = _Conf(conf)
        args = ["-w", "256", "-r", str(data_port), "-a", str(approach), "-m", "1", "-g", "/tmp",
                "-s", str(max_buf_kb)]
        n = native()
        self.bridge = n.Bridge(True, args, log_level, fetch_over=self._fetch_over, data_from_uda=self._data,
                               get_conf=self._conf, log=lambda m, s: self.logs.append((s, m)),
                               failure=self._failure)
        params = [str(num_maps), job_id, reduce_task_id, str(lpq_size), str(max_buf_kb * 1024),
                  str(min_buf_kb * 1024), key_class, CODEC_CLASSES.get(codec, codec) or "null",
                  str(comp_block_size), str(shuffle_mem), str(len(local_dirs)), *local_dirs]
        self.bridge.do_command(n.form_cmd(INIT, params))

    # ------------------------------------------------------------------ callbacks (native threads)
    def _fetch_over(self):
        self.fetch_over_calls += 1
        self.maps_reported = min(self.num_maps, self.maps_reported + PROGRESS_REPORT_LIMIT)

    def _data(self, buf: memoryview):
        # `buf` is a view of the native buffer, valid only during this call (like the DirectByteBuffer
        # J2CQueue copies from); the reader copies the records out
        self.bytes += len(buf)
        self.buffers += 1
        if self.validator is not None:
            self.validator.feed(buf)
        if self.reader is not None:
            self.reader.feed(buf)
            if self.reader.eof:
                self._done.set()
        elif len(buf) >= 2 and bytes(buf[-2:]) == b"\xff\xff" and native().buffer_ends_with_eof(buf) == 1:
            # (a record's own bytes may end in 0xFF 0xFF: only a walk of the framing tells the marker)
            self._done.set()
        return 0

    def _failure(self, reason: str):
        self.failure_calls += 1
        self.failure = reason
        self._done.set()

    # ------------------------------------------------------------------ Java-side API
    def fetch(self, host: str, job_id: str, map_attempt: str, partition: int) -> None:
        self.bridge.do_command(native().form_cmd(FETCH, [host, job_id, map_attempt, str(partition)]))

    def wait(self, timeout: float = 120.0):
        if not self._done.wait(timeout):
            raise TimeoutError("reduce task did not finish")
        if self.failure is not None:
            raise UdaFallback(self.failure)
        return self.reader.records if self.reader is not None else None

    def close(self) -> dict:
        import json
        self.bridge.reduce_exit()
        return json.loads(self.bridge.stats())


def run_reduce(provider_host: str, job_id: str, map_ids: list[str], partition: int, key_class: str,
               **kw) -> tuple[list, dict, "UdaConsumer"]:
    """Convenience: one reducer fetching `partition` of every map, returning (records, stats, consumer)."""
    timeout = kw.pop("timeout", 120.0)
    c = UdaConsumer(len(map_ids), job_id, f"attempt_{job_id}_r_{partition:06d}_0", key_class, **kw)
    t0 = time.perf_counter()
    for m in map_ids:
        c.fetch(provider_host, job_id, m, partition)
    recs = c.wait(timeout)
    st = c.close()
    st["wall_s"] = time.perf_counter() - t0
    return recs, st, c
