"""The 8-rank multi-rank schedule again at the end of the GPU tier, in a process that has run every
other GPU test first (pooled streams, workspaces and rings of earlier tasks alive), several fresh groups
of two validated steps each. Every round is checked where it can go wrong: received slices and own cells
before and after the merge, the merged output against its inputs' plan-time checksums, the output slot
before its D2H and the bytes the consumers received (StepStats.diag names the first bad round)."""
import os

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,maps,rounds,reducers", [(8, 2, 16, 1), (8, 2, 4, 2)])
def test_multirank_schedule_repeated_groups(require_gpu, world, maps, rounds, reducers):
    from uda_amd.models.terasort import TeraSortConfig, check_stats, make_local_group, run_collective
    from uda_amd.utils.ifile import J2CQueueReader

    groups = int(os.environ.get("UDA_MULTIRANK_GROUPS", "4"))
    for g in range(groups):
        cfg = TeraSortConfig(rows_per_gpu=12000 * maps, maps_per_rank=maps, rounds=rounds, reducers=reducers,
                             validate=True, sample_every=64, kv_buf_bytes=64 << 10, d2h_piece_bytes=256 << 10,
                             check_delivery=True)
        jobs, ck, rec = make_local_group(world, cfg, group=f"rep{world}{rounds}{reducers}g{g}")
        readers = [[J2CQueueReader(max_len=64 << 10) for _ in range(reducers)] for _ in range(world)]
        for d in range(world):
            jobs[d].set_python_sink(lambda r, b, d=d: readers[d][r].feed(b), True)
        for _ in range(2):
            stats = run_collective(jobs, lambda j: j.run_step(True))
            for d, st in enumerate(stats):
                check_stats(st, rec[d], ck[d], jobs[d].reducer_records())
                assert st["merge_errors"] == 0 and st["delivery_errors"] == 0 and st["pre_d2h_errors"] == 0
            for d in range(world):
                for r in readers[d]:
                    r.records.clear()
                    r.eof = False
        del jobs
