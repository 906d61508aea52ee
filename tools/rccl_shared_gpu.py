"""RCCL data plane with `world` ranks sharing ONE GPU (run under torch.distributed.run): every rank's
ShuffleJob uses device 0. Each rank prints one JSON line with its validated step stats.

Result on the one-GPU boxes (profiles/r2_rccl_shared_gpu.log): this RCCL build refuses two ranks on one
device (ncclCommInitRank: invalid usage), so the RCCL exchange itself needs a multi-GPU node; the run
still exercises the multi-rank bootstrap up to the communicator (it found a GIL bug in init_comm).

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 \
      tools/rccl_shared_gpu.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from uda_amd.models.terasort import TeraSortConfig, TeraSortShuffle  # noqa: E402
from uda_amd.parallel.dist import init_from_env  # noqa: E402


def main():
    ctx = init_from_env()
    cfg = TeraSortConfig(rows_per_gpu=int(os.environ.get("ROWS", "400000")), maps_per_rank=4, rounds=4, reducers=2,
                         validate=True, sample_every=64, kv_buf_bytes=64 << 10, d2h_piece_bytes=1 << 20)
    j = TeraSortShuffle(ctx, cfg, device=0)
    j.setup()
    out = []
    for step in range(2):
        st = j.step(validate=True)
        j.check(st)
        out.append({k: st[k] for k in ("records", "exchange_errors", "order_errors", "bytes_sent", "validated")
                    if k in st})
    print(json.dumps({"rank": ctx.rank, "world": ctx.world, "exchange": j.job.exchange_name
                      if hasattr(j.job, "exchange_name") else None, "steps": out}), flush=True)
    ctx.barrier()
    ctx.close()


if __name__ == "__main__":
    main()
