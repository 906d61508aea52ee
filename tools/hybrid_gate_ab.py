"""A/B of the GPU hybrid (LPQ/RPQ) NetMerger path with and without the GPU merge admission gate
(mapred.uda.gpu.max.concurrent.merges), secondary-sort data as in benchmarks/run_configs.py netmerger."""
import json
import sys
import time

sys.path.insert(0, ".")
from uda_amd import native  # noqa: E402
from uda_amd.bridge import UdaConsumer, UdaProvider  # noqa: E402
from uda_amd.utils.datagen import TEXT  # noqa: E402
from uda_amd.utils.mof import encode_partitions  # noqa: E402

maps, gb = 64, 2.0
rows = int(gb * 1e9 / 100 / maps)
runs = native().generate_runs("secondary", maps, 1, rows, 9)
prov = UdaProvider()
total = 0
for m, parts in enumerate(runs):
    data, index = encode_partitions(parts)
    total += len(data) - 2
    prov.add_mof_memory("job_ab", f"attempt_ab_m_{m:06d}_0", data, index)
res = {}
i = 0
for rep in range(3):
    for slots in (0, 6):
        conf = {"mapred.uda.merge.backend": "gpu", "mapred.uda.gpu.merge.bytes": max(1 << 20, total // 6),
                "mapred.uda.gpu.spill": "host", "mapred.uda.gpu.max.concurrent.merges": slots}
        c = UdaConsumer(maps, "job_ab", f"attempt_ab_r_{i:06d}_0", TEXT, conf=conf, keep_records=False)
        i += 1
        t0 = time.perf_counter()
        for m in range(maps):
            c.fetch("localhost", "job_ab", f"attempt_ab_m_{m:06d}_0", 0)
        c.wait(600)
        wall = time.perf_counter() - t0
        st = c.close()
        assert st["bytes_delivered"] - 2 == total
        res.setdefault(f"slots{slots}", []).append(round(total / wall / 1e9, 2))
        print(json.dumps({"slots": slots, "gbps": round(total / wall / 1e9, 2), "gate_wait_ms": st["gpu_gate_wait_ms"],
                          "fetch_ms": st["fetch_ms"], "merge_ms": st["merge_ms"]}), flush=True)
prov.close()
print(json.dumps(res), flush=True)
