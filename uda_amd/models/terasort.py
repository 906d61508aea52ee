"""TeraSort shuffle+merge on MI355X — the flagship workload.

Reference pipeline: every reducer fetches its partition of every map output
file (MOF) over RDMA, merges the sorted segments with a heap, and streams the merged records to
the Java reducer through `dataFromUda` in 1 MiB buffers.

Here (one process per GPU, W GPUs):
  * each GPU holds `maps_per_rank` TeraSort MOFs in HBM (the MOFSupplier's store),
  * each GPU hosts `reducers` reduce tasks; reducer i of GPU d owns the i-th contiguous slice of
    GPU d's key range (total order: concatenated reducer outputs are globally sorted),
  * every reducer range is cut into `rounds` cells; round q ships cell q of every reducer with an
    RCCL all-to-all over xGMI and merges it on the GPU (F2 keys -> F3 merge tree -> F4 gather,
    one merge group per reducer),
  * merged records go device -> host on the SDMA engines into a NUMA-local pinned ring and each
    reducer's consumer thread receives whole-record buffers of <= 1 MiB, the last one carrying the
    IFile EOF marker. The native J2C sink does what the Java side does with every buffer: copy it
    into a 1 MiB KVBuf and walk the records by their VInt lengths (UdaPlugin.java:369-402,498-538).
Data is synthetic and TeraGen-shaped (10-byte keys, 90-byte values, 104-byte IFile records).
"""
from __future__ import annotations

import dataclasses
import os
import sys
import secrets
import time

import numpy as np

from .._native import native
from ..parallel.dist import DistContext
from ..parallel.plan import round_bounds

RECORD_BYTES = 104  # IFile record: VInt(11) VInt(91) Text(10) Text(90)
TERAGEN_ROW_BYTES = 100


@dataclasses.dataclass
class TeraSortConfig:
    rows_per_gpu: int = 1_250_000_000   # 1e10 rows (1 TB TeraGen) over 8 GPUs
    maps_per_rank: int = 32
    rounds: int = 16
    seed: int = 0x5EED
    kv_buf_bytes: int = 1 << 20         # J2CQueue kv_buf_size (UdaPlugin.java:168)
    reducers: int = 1                   # reduce tasks per GPU
    d2h_piece_bytes: int = 128 << 20
    pinned_slots: int = 16
    d2h_engines: int = 1
    d2h: str = "sdma"                   # "sdma" (explicit copy engines) or "hip" (hipMemcpyAsync)
    deliver_host: bool = True
    validate: bool = False
    sample_every: int = 4096
    store: str = "hbm"                  # "hbm", "host" (pinned DRAM) or "disk" (MOF files, jobs > HBM + DRAM)
    local_dirs: str = "/tmp"            # store="disk": comma-separated directories for the MOF files
    replan: bool = False                # every step recomputes the cell splits and exchanges the counts
    map_sort: bool = False              # setup: unsorted map input sorted on the device (F8 radix sort)
    check_delivery: bool = False        # validate steps: checksum every round output before its D2H and as received
    exchange: str = "ipc"               # world > 1: "ipc" (shared-memory control + hipIpc pulls) or "rccl"


class TeraSortShuffle:
    def __init__(self, ctx: DistContext, cfg: TeraSortConfig, device: int | None = None):
        self.ctx = ctx
        self.cfg = cfg
        self.device = ctx.local_rank if device is None else device
        n = native()
        records_per_map = max(1, cfg.rows_per_gpu // cfg.maps_per_rank)
        self.records_per_map = records_per_map
        self.job = n.ShuffleJob(dict(
            device=self.device, rank=ctx.rank, world=ctx.world,
            maps_per_rank=cfg.maps_per_rank, records_per_map=records_per_map,
            rounds=cfg.rounds, reducers=cfg.reducers, seed=cfg.seed, kv_buf_bytes=cfg.kv_buf_bytes,
            d2h_piece_bytes=cfg.d2h_piece_bytes, pinned_slots=cfg.pinned_slots,
            d2h_engines=cfg.d2h_engines, d2h=cfg.d2h, deliver_host=cfg.deliver_host,
            validate=cfg.validate, store=cfg.store, local_dirs=cfg.local_dirs, replan=cfg.replan,
            map_sort=cfg.map_sort, check_delivery=cfg.check_delivery))
        self.sink = n.J2CSink(cfg.reducers, cfg.kv_buf_bytes)
        self.expected_checksum = None
        self.expected_records = None
        self.setup_s = {}

    def setup(self) -> None:
        n = native()
        t0 = time.perf_counter()
        if self.ctx.world > 1:
            if self.cfg.exchange == "ipc" and not self._ipc_preflight():
                # every rank saw the same verdict (all-gathered), so all switch together: the shuffle runs
                # over RCCL, and the reason stays in the job's record (ipc_fallback, the bench JSON).
                # UDA_IPC_FALLBACK=0 stops the job instead.
                if os.environ.get("UDA_IPC_FALLBACK", "1") == "0":
                    raise RuntimeError(f"IPC exchange preflight failed ({self.ipc_fallback}); the job stops here "
                                       "(UDA_IPC_FALLBACK=0)")
                if self.ctx.rank == 0:
                    print(f"uda: IPC exchange preflight failed, shuffling over RCCL ({self.ipc_fallback})",
                          file=sys.stderr, flush=True)
                self.cfg.exchange = "rccl"
            if self.cfg.exchange == "ipc":
                name = f"uda.{os.getpid()}.{secrets.token_hex(6)}".encode() if self.ctx.rank == 0 else None
                self.job.init_ipc(self.ctx.broadcast_bytes(name).decode())
            elif self.cfg.exchange == "rccl":
                uid = n.nccl_unique_id() if self.ctx.rank == 0 else None
                uid = self.ctx.broadcast_bytes(uid)
                self.job.init_comm(uid)
            else:
                raise ValueError(f"unknown exchange {self.cfg.exchange!r}")
        t1 = time.perf_counter()
        self.job.generate()
        t2 = time.perf_counter()
        # sample keys -> per-destination quantile bounds (all ranks agree)
        local = self.job.sample_keys(self.cfg.sample_every)
        gathered = self.ctx.all_gather_object([np.asarray(a) for a in local])
        per_dest = []
        for d in range(self.ctx.world):
            parts = [g[d] for g in gathered if g[d].size]
            per_dest.append(np.concatenate(parts) if parts else np.zeros((0, 2), np.uint64))
        bounds = round_bounds(per_dest, self.cfg.rounds * self.cfg.reducers)
        self.job.set_bounds(np.ascontiguousarray(bounds.reshape(-1)))
        self.job.plan()
        t3 = time.perf_counter()
        # expected per-reducer checksum/records for validation
        ck = self.ctx.sum_u64(self.job.local_dest_checksums())
        rec = self.ctx.sum_u64(self.job.local_dest_records())
        self.expected_checksum = ck[self.ctx.rank]
        self.expected_records = rec[self.ctx.rank]
        self.job.set_j2c_sink(self.sink)
        self.setup_s = dict(comm_init=t1 - t0, generate=t2 - t1, plan=t3 - t2)

    def _ipc_preflight(self) -> bool:
        """Before the job commits to the IPC exchange, the shuffle's own pattern on a small scale: every
        rank exports one device allocation larger than 4 GiB (a map-output store is one multi-GB export,
        padded by ipc_safe_bytes) holding 16 slices per peer of the production slice size spread up to
        its end, every peer maps it over hipIpc and pulls its slices with the batched copy kernel, 2
        rounds, every byte checked (exchange_probe). All ranks all-gather the outcome, so they agree;
        on failure the job stops with the reason (`ipc_fallback`). UDA_IPC_PREFLIGHT=0 skips it."""
        self.ipc_fallback = None
        if os.environ.get("UDA_IPC_PREFLIGHT", "1") == "0":
            return True
        w, r, c = self.ctx.world, self.ctx.rank, self.cfg
        # a round's slice: one map output's cell for one reducer (store / (maps x world x reducers x rounds))
        store = c.rows_per_gpu * RECORD_BYTES
        slice_bytes = store // max(1, c.maps_per_rank * w * c.reducers * c.rounds)
        slice_bytes = int(min(64 << 20, max(4096, slice_bytes))) // 104 * 104
        size = lambda f, t: [slice_bytes + 104 * ((f + t + i) % 7) for i in range(16)]  # noqa: E731
        send = [size(r, p) if p != r else [] for p in range(w)]
        recv = [size(p, r) if p != r else [] for p in range(w)]
        export = int(os.environ.get("UDA_IPC_PREFLIGHT_EXPORT", str((4 << 30) + (256 << 20))))
        name = f"udapre.{os.getpid()}.{secrets.token_hex(6)}".encode() if r == 0 else None
        name = self.ctx.broadcast_bytes(name).decode()
        try:
            err = native().ipc_exchange_probe(name, r, w, send, recv, False, 2, self.device, export)
        except Exception as e:  # noqa: BLE001 - reported to every rank below
            err = f"{type(e).__name__}: {e}"
        errs = self.ctx.all_gather_object(err)
        bad = [f"rank {i}: {e}" for i, e in enumerate(errs) if e]
        if bad:
            self.ipc_fallback = "; ".join(bad)[:500]
            if r == 0:
                print(f"uda: IPC exchange preflight failed ({self.ipc_fallback})", file=sys.stderr, flush=True)
            return False
        return True

    def step(self, validate: bool | None = None) -> dict:
        """One shuffle+merge+deliver pass. Every step checks what the consumers parsed (records per
        reducer, framing, EOF); validate=True also runs the device order/checksum/exchange checks."""
        if self.sink is not None and self.cfg.deliver_host:
            self.sink.reset()
        st = self.job.run_step(self.cfg.validate if validate is None else validate)
        if self.sink is not None and self.cfg.deliver_host:
            self.sink.flush()  # the reduce tasks' threads walked every delivered KVBuf
            st["consumer_records"] = [self.sink.records(i) for i in range(self.cfg.reducers)]
            st["consumer_errors"] = [self.sink.error(i) for i in range(self.cfg.reducers)]
            st["consumer_eof"] = [self.sink.eof(i) for i in range(self.cfg.reducers)]
        return st

    def drop_sink(self) -> None:
        """Ablation: delivered buffers are released unread (no consumer work)."""
        self.sink = None
        self.job.clear_sink()

    def use_python_sink(self, fn, with_reducer: bool = False) -> None:
        """Deliver to a Python callable instead of the native J2C sink (tests)."""
        self.sink = None
        self.job.set_python_sink(fn, with_reducer)

    def check(self, stats: dict) -> None:
        """Raise if a step lost, duplicated, corrupted or mis-ordered records."""
        check_stats(stats, self.expected_records, self.expected_checksum, self.job.reducer_records())


def check_stats(stats: dict, expected_records: int, expected_checksum: int, reducer_records) -> None:
    if stats["records"] != expected_records:
        raise AssertionError(f"records {stats['records']} != expected {expected_records}")
    if stats["bad_layout"]:
        raise AssertionError("non-TeraSort record layout seen by the merge")
    if "consumer_records" in stats:
        if list(stats["consumer_records"]) != list(reducer_records):
            raise AssertionError(f"consumers parsed {stats['consumer_records']} records, expected {reducer_records}")
        if any(stats["consumer_errors"]):
            raise AssertionError(f"consumer framing errors {stats['consumer_errors']}")
        if not all(stats["consumer_eof"]):
            raise AssertionError("a reducer did not receive its EOF marker")
    if stats["validated"]:
        if stats["order_errors"] != 0:
            raise AssertionError(f"{stats['order_errors']} out-of-order records")
        if stats["exchange_errors"] != 0:
            raise AssertionError(f"{stats['exchange_errors']} received slices differ from what their sender sent")
        for k in ("pre_merge_errors", "own_errors", "merge_errors", "pre_d2h_errors", "delivery_errors"):
            if stats.get(k, 0) > 0:
                raise AssertionError(f"{k} {stats[k]}: {stats.get('diag', '')}")
        if stats["checksum"] != expected_checksum:
            raise AssertionError("checksum mismatch " + stats.get("diag", ""))


def make_local_group(world: int, cfg: TeraSortConfig, device: int = 0, group: str = "local"):
    """Single-process rehearsal of a `world`-rank shuffle: every rank is a ShuffleJob on `device`
    driven from its own thread, exchanging rounds through device memcpys with the same pack /
    all-to-all-v schedule as the RCCL path. Returns (jobs, expected_checksums, expected_records)."""

    n = native()
    records_per_map = max(1, cfg.rows_per_gpu // cfg.maps_per_rank)
    jobs = [n.ShuffleJob(dict(
        device=device, rank=r, world=world, maps_per_rank=cfg.maps_per_rank,
        records_per_map=records_per_map, rounds=cfg.rounds, reducers=cfg.reducers, seed=cfg.seed,
        kv_buf_bytes=cfg.kv_buf_bytes, d2h_piece_bytes=cfg.d2h_piece_bytes, pinned_slots=cfg.pinned_slots,
        d2h_engines=cfg.d2h_engines, d2h=cfg.d2h, deliver_host=cfg.deliver_host, validate=cfg.validate,
        local_group=group, store=cfg.store, local_dirs=cfg.local_dirs, replan=cfg.replan,
        map_sort=cfg.map_sort, check_delivery=cfg.check_delivery))
        for r in range(world)]
    for j in jobs:
        j.init_local()
        j.generate()
    local = [j.sample_keys(cfg.sample_every) for j in jobs]
    per_dest = []
    for d in range(world):
        parts = [np.asarray(s[d]) for s in local if np.asarray(s[d]).size]
        per_dest.append(np.concatenate(parts) if parts else np.zeros((0, 2), np.uint64))
    bounds = np.ascontiguousarray(round_bounds(per_dest, cfg.rounds * cfg.reducers).reshape(-1))
    for j in jobs:
        j.set_bounds(bounds)
    run_collective(jobs, lambda j: j.plan())
    ck = [sum(j.local_dest_checksums()[d] for j in jobs) % (1 << 64) for d in range(world)]
    rec = [sum(j.local_dest_records()[d] for j in jobs) for d in range(world)]
    return jobs, ck, rec


def run_collective(jobs, fn):
    """Call fn(job) on every rank concurrently (collective operations need all ranks)."""
    import threading

    out = [None] * len(jobs)
    err = []

    def work(i):
        try:
            out[i] = fn(jobs[i])
        except BaseException as e:  # noqa: BLE001
            err.append(e)

    ts = [threading.Thread(target=work, args=(i,)) for i in range(len(jobs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if err:
        raise err[0]
    return out
