"""Stress the multi-rank shuffle schedule (ranks as threads of one process sharing one GPU) and
localise any checksum mismatch per (round, reducer) and per stage.

Every validated step checks, per round: the received slices and own cells before and after the merge,
the merged output against the sum of its inputs' plan-time checksums and (--check-delivery) the output
slot right before its D2H and the bytes each consumer received. A failing step prints
StepStats.diag (the first mismatching round/reducer of each kind).

    python tools/multirank_stress.py --world 8 --maps 2 --rounds 16 --steps 40 --idle-streams 24
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--maps", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=16)
    ap.add_argument("--reducers", type=int, default=1)
    ap.add_argument("--rows-per-map", type=int, default=12000)
    ap.add_argument("--steps", type=int, default=20, help="validated steps per group")
    ap.add_argument("--groups", type=int, default=1, help="fresh groups (new jobs, new plans)")
    ap.add_argument("--idle-streams", type=int, default=0, help="idle streams held alive before the jobs start")
    ap.add_argument("--noise-streams", type=int, default=0, help="extra streams kept busy with device copies")
    ap.add_argument("--noise-bytes", type=int, default=8 << 20)
    ap.add_argument("--python-sink", type=int, default=1, help="1: consumers feed Python readers (as the test)")
    ap.add_argument("--check-delivery", type=int, default=1)
    ap.add_argument("--stop-on-fail", type=int, default=0)
    ap.add_argument("--old-memset", type=int, default=0,
                    help="1: zero the generation checksums with a null-stream hipMemset (the r5 code) to show the race; "
                         "2: also the DeviceMerger's null-stream memsets without the stream sync (r5 exactly)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    if a.old_memset:
        os.environ["UDA_GEN_NULL_STREAM_MEMSET"] = str(a.old_memset)
    from uda_amd import native
    from uda_amd.models.terasort import TeraSortConfig, make_local_group, run_collective
    from uda_amd.utils.ifile import J2CQueueReader

    n = native()
    if a.idle_streams:
        n.hold_idle_streams(0, a.idle_streams, 0)
    if a.noise_streams:
        n.start_gpu_noise(0, a.noise_streams, a.noise_bytes)
    keys = ("records", "order_errors", "exchange_errors", "pre_merge_errors", "own_errors", "merge_errors",
            "pre_d2h_errors", "delivery_errors")
    fails = []
    steps = 0
    t0 = time.time()
    for g in range(a.groups):
        cfg = TeraSortConfig(rows_per_gpu=a.rows_per_map * a.maps, maps_per_rank=a.maps, rounds=a.rounds,
                             reducers=a.reducers, validate=True, sample_every=64, kv_buf_bytes=64 << 10,
                             d2h_piece_bytes=256 << 10, check_delivery=bool(a.check_delivery))
        try:
            jobs, ck, rec = make_local_group(a.world, cfg, group=f"stress{g}")
        except RuntimeError as e:  # the plan's self-check: generation checksum != store content
            fails.append({"group": g, "step": -1, "setup_error": str(e)[:300]})
            print("SETUP FAIL", json.dumps(fails[-1]), flush=True)
            continue
        if a.python_sink:
            readers = [[J2CQueueReader(max_len=64 << 10) for _ in range(a.reducers)] for _ in range(a.world)]
            for d in range(a.world):
                jobs[d].set_python_sink(lambda r, b, d=d: readers[d][r].feed(b), True)
        for s in range(a.steps):
            stats = run_collective(jobs, lambda j: j.run_step(True))
            steps += 1
            for d, st in enumerate(stats):
                bad = (st["checksum"] != ck[d] or st["records"] != rec[d] or
                       any(st[k] > 0 for k in keys if k != "records"))
                if bad:
                    f = {"group": g, "step": s, "rank": d, "checksum_ok": st["checksum"] == ck[d],
                         "diag": st["diag"], **{k: st[k] for k in keys}}
                    fails.append(f)
                    print("FAIL", json.dumps(f), flush=True)
            if a.python_sink:  # drop what the readers parsed (memory), keep them attached
                for d in range(a.world):
                    for r in readers[d]:
                        r.records.clear()
                        r.eof = False
            print(f"group {g} step {s}: {'fail' if fails and fails[-1]['step'] == s and fails[-1]['group'] == g else 'ok'}"
                  f" ({time.time() - t0:.1f}s)", flush=True)
            if fails and a.stop_on_fail:
                break
        del jobs
        if fails and a.stop_on_fail:
            break
    noise_ops = n.stop_gpu_noise() if a.noise_streams else 0
    summary = {"steps": steps, "noise_copies": noise_ops, "failed_rank_steps": len(fails), "fails": fails[:20],
               "config": vars(a), "seconds": round(time.time() - t0, 1)}
    print(json.dumps(summary), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
