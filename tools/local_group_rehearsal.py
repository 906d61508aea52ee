"""Larger single-GPU rehearsal of the multi-rank shuffle schedule: `world` ranks share one GPU and
exchange through in-process pulls (same plans, slots, rounds and validation as the RCCL path).
Reports per-step time and checks every rank's records, checksum and exchanged slices."""
import argparse
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/", 2)[0])
import torch  # noqa: F401,E402
from uda_amd import native  # noqa: E402
from uda_amd.models.terasort import TeraSortConfig, check_stats, make_local_group, run_collective  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--rows-per-rank", type=int, default=20_000_000)
ap.add_argument("--reducers", type=int, default=16)
ap.add_argument("--rounds", type=int, default=16)
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--no-map-sort", action="store_true", help="generate sorted runs directly (bench --no-map-sort)")
a = ap.parse_args()
cfg = TeraSortConfig(rows_per_gpu=a.rows_per_rank, maps_per_rank=32, rounds=a.rounds, reducers=a.reducers,
                     validate=True, map_sort=not a.no_map_sort)
t = time.perf_counter()
jobs, ck, rec = make_local_group(a.world, cfg, group="rehearsal")
setup = time.perf_counter() - t
sinks = []
for j in jobs:
    s = native().J2CSink(a.reducers, cfg.kv_buf_bytes)
    j.set_j2c_sink(s)
    sinks.append(s)
times = []
for step in range(a.steps):
    t = time.perf_counter()
    stats = run_collective(jobs, lambda j: j.run_step(True))
    times.append(time.perf_counter() - t)
    for d, st in enumerate(stats):
        check_stats(st, rec[d], ck[d], jobs[d].reducer_records())
        assert st["exchange_errors"] == 0 and st["order_errors"] == 0, st
    for s in sinks:
        s.reset()
total = sum(rec) * 104
print(json.dumps({"world": a.world, "gb_total": round(total / 1e9, 2), "setup_s": round(setup, 1),
                  "step_s": [round(x, 3) for x in times], "exchange": jobs[0].exchange_name,
                  "validated": True}))
