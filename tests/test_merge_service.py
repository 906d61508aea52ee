"""CPU tier: the node merge service driven through the C ABI in one process (a provider hosting the
service, reduce tasks as its clients through uda_start with mapred.uda.gpu.merge.service), so host
sanitizers (tools/run_sanitizers.py: ASan, TSan) see both sides of the socket protocol. The
multi-process shape (fresh task processes) is covered by tests/test_reduce_task_exe.py.

Reference: the NetMerger runs inside each reduce task's JVM (src/UdaBridge.cc:187-263); here it can run
in the provider process (csrc/service/merge_service.h) with the same host contract."""
import socket
import threading

from uda_amd.bridge import UdaConsumer, UdaProvider
from uda_amd.utils import datagen
from uda_amd.utils.mof import encode_partitions


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_service_hosted_tasks_in_one_process(native, tmp_path):
    """Four reduce tasks at once, each a client of the service in the same process; records, order and
    the fetch-over / stats callbacks as with in-process tasks."""
    port = _port()
    path = str(tmp_path / "svc.sock")
    prov = UdaProvider(transport="tcp", data_port=port,
                       conf={"mapred.uda.provider.bind.address": "127.0.0.1", "mapred.uda.gpu.merge.service": path})
    try:
        job = "job_9_0001"
        maps = datagen.terasort(num_maps=6, reducers=4, rows_per_map=800, seed=91)
        ids = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_{job}_m_{i:06d}_0"
            data, index = encode_partitions(parts, None)
            prov.add_mof_memory(job, mid, data, index)
            ids.append(mid)
        results = {}

        def run(r):
            c = UdaConsumer(len(ids), job, f"attempt_{job}_r_{r:06d}_0", datagen.TEXT, transport="tcp",
                            data_port=port, kv_buf_size=32 << 10,
                            conf={"mapred.uda.merge.backend": "cpu", "mapred.uda.gpu.merge.service": path})
            for m in ids:
                c.fetch("127.0.0.1", job, m, r)
            recs = c.wait(60)
            results[r] = (recs, c.close(), c.fetch_over_calls)

        ts = [threading.Thread(target=run, args=(r,)) for r in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for r in range(4):
            recs, st, fo = results[r]
            want = sorted(kv for m in maps for kv in m[r])
            assert recs == want
            assert st.get("merge_service") is True and st["maps_fetched"] == 6 and fo >= 1, st
    finally:
        prov.close()


def test_unreachable_service_merges_in_process(native, tmp_path):
    port = _port()
    prov = UdaProvider(transport="tcp", data_port=port, conf={"mapred.uda.provider.bind.address": "127.0.0.1"})
    try:
        job = "job_9_0002"
        maps = datagen.terasort(num_maps=3, reducers=1, rows_per_map=500, seed=92)
        ids = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_{job}_m_{i:06d}_0"
            data, index = encode_partitions(parts, None)
            prov.add_mof_memory(job, mid, data, index)
            ids.append(mid)
        c = UdaConsumer(3, job, f"attempt_{job}_r_000000_0", datagen.TEXT, transport="tcp", data_port=port,
                        conf={"mapred.uda.merge.backend": "cpu",
                              "mapred.uda.gpu.merge.service": str(tmp_path / "nobody.sock")})
        for m in ids:
            c.fetch("127.0.0.1", job, m, 0)
        assert c.wait(60) == sorted(kv for m in maps for kv in m[0])
        st = c.close()
        assert "merge_service" not in st
        assert any("merge service unavailable" in msg for _, msg in c.logs)
    finally:
        prov.close()
