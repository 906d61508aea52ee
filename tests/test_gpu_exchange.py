"""GPU: the exchange backends under the NCCL point-to-point rules, and the multi-process shuffle.

* LocalExchange (threads) and IpcExchange (real processes, hipIpc + shared-memory control plane)
  with hand-made plans: matched plans move every byte; a send/recv count or size mismatch and a
  host-pinned source are refused (the rules RCCL imposes; reference: the pairwise RDMA
  WRITE/ACK of src/DataNet/RDMAServer.cc:537-631 and RDMAClient.cc:559-600).
* `bench.py --gpus N --one-gpu --exchange ipc`: N rank processes on GPU 0 run the whole TeraSort
  shuffle (counts all-to-all, per-round pulls from the peers' HBM, merge, delivery) and must
  report validated with zero exchange-checksum errors, for the HBM, pinned-DRAM and disk stores.
"""
import json
import multiprocessing as mp
import os
import secrets
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _plan(world, sizes):
    """sizes(from, to) -> list of slice sizes; returns (send[r][p], recv[r][p])."""
    send = [[sizes(r, p) if p != r else [] for p in range(world)] for r in range(world)]
    recv = [[sizes(p, r) if p != r else [] for p in range(world)] for r in range(world)]
    return send, recv


def _sizes(f, t):
    if (f + t) % 3 == 2:
        return []  # a pair that exchanges nothing
    return [4096 * (1 + (f * 7 + t * 3 + i) % 5) + 104 * i for i in range(1 + (f + 2 * t) % 4)]


def test_local_exchange_matched(require_gpu, native):
    send, recv = _plan(4, _sizes)
    assert native.local_exchange_probe(4, send, recv, rounds=3) == [""] * 4


def test_local_exchange_refuses_count_mismatch(require_gpu, native):
    send, recv = _plan(3, _sizes)
    send[0][1] = send[0][1] + [1024]  # rank 0 sends one slice more than rank 1 posts
    errs = native.local_exchange_probe(3, send, recv)
    assert "pairing" in errs[1], errs
    assert all(e for e in errs), errs  # the group aborts: nobody completes silently


def test_local_exchange_refuses_size_mismatch(require_gpu, native):
    send, recv = _plan(2, lambda f, t: [8192, 4096])
    recv[1][0] = [8192, 4000]
    errs = native.local_exchange_probe(2, send, recv)
    assert "4000" in errs[1] and "bytes" in errs[1], errs


def test_local_exchange_refuses_host_source(require_gpu, native):
    send, recv = _plan(2, lambda f, t: [65536])
    errs = native.local_exchange_probe(2, send, recv, host_source=True)
    assert any("not device memory" in e for e in errs), errs


def _ipc_rank(name, rank, world, send, recv, host_source, rounds, export, q):
    import uda_amd
    q.put((rank, uda_amd.native().ipc_exchange_probe(name, rank, world, send, recv, host_source, rounds, 0, export)))


def _run_ipc(world, send, recv, host_source=False, rounds=1, export=0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"udaprobe.{os.getpid()}.{secrets.token_hex(4)}"
    ps = [ctx.Process(target=_ipc_rank, args=(name, r, world, send[r], recv[r], host_source, rounds, export, q))
          for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(world):
        r, v = q.get(timeout=180)
        out[r] = v
    for p in ps:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    return [out[r] for r in range(world)]


def test_ipc_exchange_matched_processes(require_gpu):
    send, recv = _plan(3, _sizes)
    assert _run_ipc(3, send, recv, rounds=4) == [""] * 3


def test_ipc_preflight_shape_over_a_store_sized_export(require_gpu):
    """The job's preflight shape: each rank exports one allocation larger than 4 GiB (padded out of
    the hipIpc-hanging size range) with production-size slices spread up to its end; the peers map
    it and pull every slice with the batched copy kernel, every byte checked."""
    slice_bytes = (2 << 20) // 104 * 104
    send, recv = _plan(2, lambda f, t: [slice_bytes + 104 * i for i in range(16)])
    assert _run_ipc(2, send, recv, rounds=2, export=(4 << 30) + (256 << 20)) == [""] * 2


def test_ipc_exchange_refuses_mismatch_and_host_source(require_gpu):
    send, recv = _plan(2, lambda f, t: [8192, 4096])
    recv[0][1] = [8192]
    errs = _run_ipc(2, send, recv)
    assert "pairing" in errs[0], errs
    assert errs[1], errs  # the peer is woken by the abort
    send, recv = _plan(2, lambda f, t: [65536])
    errs = _run_ipc(2, send, recv, host_source=True)
    assert any("not device memory" in e for e in errs), errs


def _bench(*extra, timeout=600):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
           "--d2h-piece-mb", "8", "--pinned-slots", "4", *extra]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line), r.stderr


@pytest.mark.parametrize("ranks", [2, 4])
def test_bench_multiprocess_ipc_one_gpu(require_gpu, ranks):
    out, err = _bench("--gpus", str(ranks), "--one-gpu", "--exchange", "ipc", "--rows-per-gpu", "2000000",
                      "--maps-per-gpu", "4", "--reducers", "4", "--rounds", "3")
    assert out["validated"] is True and out["exchange_errors"] == 0, (out, err[-2000:])
    assert out["ranks"] == ranks and out["exchange"] == "ipc"
    assert all(b > 0 for b in out["bytes_sent_per_rank"])
    assert out["config"]["global_batch"] == 2000000 * ranks


@pytest.mark.parametrize("store", ["host", "disk"])
def test_bench_multiprocess_ipc_spill_tiers(require_gpu, tmp_path, store):
    extra = ["--local-dirs", f"{tmp_path}"] if store == "disk" else []
    out, err = _bench("--gpus", "2", "--one-gpu", "--exchange", "ipc", "--store", store, "--rows-per-gpu", "1000000",
                      "--maps-per-gpu", "3", "--reducers", "2", "--rounds", "4", *extra)
    assert out["validated"] is True and out["exchange_errors"] == 0, (out, err[-2000:])
    assert out["breakdown_ms_rank0"]["stage_ms"] > 0
    assert store in out["config"]["store"].lower() or "disk" in out["config"]["store"]
