"""One-process-per-GPU bootstrap.

The control plane (rendezvous, barriers, small all-gathers of key samples/checksums) runs over
torch.distributed (gloo, CPU); the data plane is the engine's own RCCL communicator over xGMI,
bootstrapped here with an ncclUniqueId broadcast from rank 0 (reference analogue: RDMA-CM
connection setup, src/DataNet/RDMAClient.cc:215-356).
"""
from __future__ import annotations

import dataclasses
import datetime
import os

import torch
import torch.distributed as dist


@dataclasses.dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    initialized: bool = False

    @property
    def is_distributed(self) -> bool:
        return self.world > 1

    def barrier(self) -> None:
        if self.initialized:
            dist.barrier()

    def broadcast_bytes(self, data: bytes | None) -> bytes:
        if not self.initialized:
            assert data is not None
            return data
        obj = [data]
        dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def all_gather_object(self, obj):
        if not self.initialized:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj)
        return out

    def max_float(self, x: float) -> float:
        if not self.initialized:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_u64(self, values: list[int]) -> list[int]:
        """Sum unsigned 64-bit values across ranks modulo 2**64."""
        if not self.initialized:
            return [v % (1 << 64) for v in values]
        gathered = self.all_gather_object([int(v) for v in values])
        return [sum(g[i] for g in gathered) % (1 << 64) for i in range(len(values))]

    def close(self) -> None:
        if self.initialized and dist.is_initialized():
            dist.destroy_process_group()
            self.initialized = False


def init_from_env(backend: str = "gloo", timeout_s: int = 1800) -> DistContext:
    """Read RANK/LOCAL_RANK/WORLD_SIZE (torchrun) and init the control-plane process group."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    ctx = DistContext(rank=rank, world=world, local_rank=local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s))
        ctx.initialized = True
    return ctx
