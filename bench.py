#!/usr/bin/env python3
"""Headline benchmark: TeraSort shuffle+merge GB/s, whole node (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W
    (N>1 is launched by torchrun: one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE from env)

One step = the whole reduce-side shuffle of a TeraSort job: every GPU's reducer receives its key
range from every GPU's map outputs (RCCL all-to-all over xGMI in key-range rounds), merges them on
the GPU and delivers the merged records to the host reducer in <=1 MiB whole-record buffers
(the `dataFromUda` contract), EOF marker included. Per-GPU data is fixed (weak scaling):
--rows-per-gpu TeraGen rows (104-byte IFile records) per GPU; the default 1.25e9 rows/GPU makes
N=8 the 1 TB TeraSort config (N=1 moves 130 GB through one GPU).

value = total partition bytes delivered on all GPUs / time per step (GB = 1e9 bytes).
Data is synthetic (TeraGen-shaped keys/values generated in HBM; see uda_amd/models/terasort.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows-per-gpu", type=int, default=1_250_000_000)
    ap.add_argument("--maps-per-gpu", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=16)
    # D2H staging: 4 x 512 MiB pinned pieces on one copy stream. Swept on MI355X
    # (profiles/r1_d2h_sweep.json): 64 MiB x6 -> 55.9 GB/s, 512 MiB x4 -> 56.7 GB/s against a
    # 57.0 GB/s single-copy PCIe roof; two copy streams contend and drop to ~22 GB/s.
    ap.add_argument("--d2h-piece-mb", type=int, default=512)
    ap.add_argument("--pinned-slots", type=int, default=4)
    ap.add_argument("--d2h-streams", type=int, default=1)
    ap.add_argument("--device-only", action="store_true",
                    help="ablation: stop after the device merge (no host delivery); not the headline")
    ap.add_argument("--validate", action="store_true", help="run one extra validated step at the end")
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args()

    import torch  # noqa: F401  (loads the HIP runtime before the native extension)

    from uda_amd.models.terasort import RECORD_BYTES, TeraSortConfig, TeraSortShuffle
    from uda_amd.parallel.dist import init_from_env

    ctx = init_from_env()
    if ctx.world != args.gpus:
        if ctx.world == 1 and args.gpus > 1:
            print(f"--gpus {args.gpus} requires a torchrun launch (WORLD_SIZE is 1)", file=sys.stderr)
            return 2
    torch.cuda.set_device(ctx.local_rank)

    cfg = TeraSortConfig(rows_per_gpu=args.rows_per_gpu, maps_per_rank=args.maps_per_gpu,
                         rounds=args.rounds, d2h_piece_bytes=args.d2h_piece_mb << 20,
                         pinned_slots=args.pinned_slots, d2h_streams=args.d2h_streams,
                         deliver_host=not args.device_only)
    job = TeraSortShuffle(ctx, cfg)
    t_setup = time.perf_counter()
    job.setup()
    t_setup = time.perf_counter() - t_setup
    if args.verbose and ctx.rank == 0:
        print(f"# setup {t_setup:.1f}s {job.setup_s} store={job.job.store_bytes/1e9:.1f}GB "
              f"max_round_records={job.job.max_round_records}", file=sys.stderr, flush=True)

    for i in range(args.warmup):
        st = job.step()
        job.check(st)
        if args.verbose and ctx.rank == 0:
            print(f"# warmup {i}: {json.dumps(st)}", file=sys.stderr, flush=True)

    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        stats.append(job.step())
    torch.cuda.synchronize()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = ctx.max_float(elapsed)
    for st in stats:
        job.check(st)

    validated = None
    if args.validate:
        job.job_validate = True
        from uda_amd.models.terasort import TeraSortConfig as _C  # noqa: F401
        vcfg = dict(cfg.__dict__)
        vcfg["validate"] = True
        vjob = TeraSortShuffle(ctx, TeraSortConfig(**vcfg))
        del job  # free HBM before the validation job allocates its own store
        vjob.setup()
        vst = vjob.step()
        vjob.check(vst)
        validated = True

    bytes_per_gpu = stats[0]["bytes_in"]
    total_bytes = sum(ctx.all_gather_object(bytes_per_gpu))
    ms_per_step = elapsed * 1000.0 / max(1, args.steps)
    gbps = total_bytes / (ms_per_step / 1000.0) / 1e9
    mean = lambda k: sum(s[k] for s in stats) / len(stats)  # noqa: E731
    if ctx.rank == 0:
        out = {
            "metric": "TeraSort shuffle+merge GB/s whole-node",
            "value": round(gbps, 3),
            "unit": "GB/s",
            "n_gpus": ctx.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bytes",
            "data": "synthetic TeraGen-shaped (10B key/90B value, 104B IFile records generated in HBM)",
            "config": {
                "model": "terasort",
                "global_batch": int(args.rows_per_gpu) * ctx.world,
                "seq_len": RECORD_BYTES,
                "parallelism": f"dp{ctx.world}",
                "rows_per_gpu": args.rows_per_gpu,
                "total_rows": args.rows_per_gpu * ctx.world,
                "maps_per_gpu": args.maps_per_gpu,
                "rounds": args.rounds,
                "shuffle": "rccl-a2a-xgmi" if ctx.world > 1 else "local (single GPU, no all-to-all)",
                "delivery": "device-only (ablation)" if args.device_only else "host dataFromUda <=1MiB buffers",
            },
            "reduce_wall_clock_s": round(ms_per_step / 1000.0, 3),
            "teragen_gbps": round(gbps * 100 / RECORD_BYTES, 3),
            "breakdown_ms_rank0": {k: round(mean(k), 2) for k in ("split_ms", "comm_ms", "merge_ms", "d2h_ms")},
            "merge_passes": stats[0]["merge_passes"],
            "buffers_per_step": stats[0]["buffers"],
            "validated": validated,
            "reference_envelope_gbps_per_node": 5.0,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
