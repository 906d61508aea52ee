"""CPU tier: uda_reduce_task, one reduce task in a process of its own (as Hadoop runs each reduce task
in its own JVM), against a MOFSupplier in another process over the TCP transport: INIT and FETCH
commands on stdin, the merged stream walked by the J2C consumer, one JSON line out.

Reference: UdaBridge startNative / doCommandNative (src/UdaBridge.cc:187-295), NetMergerMain
(src/Merger/NetMergerMain.cc:44-77), J2CQueue (plugins/shared/.../UdaPlugin.java:456-538)."""
import json
import os
import socket
import subprocess

import pytest

from uda_amd.bridge import FETCH, INIT, UdaProvider
from uda_amd.utils import datagen
from uda_amd.utils.mof import encode_partitions

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "uda_amd", "bin", "uda_reduce_task")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _task(native, port, job, ids, r, expect, backend="cpu", order=False, extra=()):
    argv = [EXE, "-D", "mapred.uda.transport=tcp", "-D", f"mapred.uda.merge.backend={backend}", *extra,
            "--expect", str(expect), "--kv-buf", str(64 << 10)] + (["--check-order"] if order else [])
    argv += ["--", "-w", "256", "-r", str(port), "-a", "1", "-m", "1", "-g", "/tmp", "-s", "1024"]
    init = native.form_cmd(INIT, [str(len(ids)), job, f"attempt_{job}_r_{r:06d}_0", "0", str(1 << 20),
                                  str(16 << 10), datagen.TEXT, "null", str(256 << 10), "0", "0"])
    lines = [init] + [native.form_cmd(FETCH, ["127.0.0.1", job, m, str(r)]) for m in ids]
    p = subprocess.run(argv, input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=120)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    return p.returncode, out


@pytest.mark.skipif(not os.access(EXE, os.X_OK), reason="uda_reduce_task not built")
def test_reduce_task_processes_against_a_provider_process(native):
    port = _port()
    prov = UdaProvider(transport="tcp", data_port=port, conf={"mapred.uda.provider.bind.address": "127.0.0.1"})
    try:
        job = "job_7_0001"
        maps = datagen.terasort(num_maps=5, reducers=2, rows_per_map=2000, seed=77)
        ids = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_{job}_m_{i:06d}_0"
            data, index = encode_partitions(parts, None)
            prov.add_mof_memory(job, mid, data, index)
            ids.append(mid)
        for r in range(2):
            want = sum(len(m[r]) for m in maps)
            rc, out = _task(native, port, job, ids, r, want, order=True)
            assert rc == 0 and out["error"] == "", out
            assert out["records"] == want and out["order_errors"] == 0
            assert out["task"]["maps_fetched"] == 5 and out["task"]["backend"] == "cpu"
            assert out["fetch_to_eof_ms"] >= 0 and out["exec_to_end_ms"] >= out["fetch_to_eof_ms"]
        rc, out = _task(native, port, job, ids, 0, 1)  # wrong expectation: the process says so
        assert rc == 1 and "expected 1" in out["error"], out
    finally:
        prov.close()


@pytest.mark.skipif(not os.access(EXE, os.X_OK), reason="uda_reduce_task not built")
def test_provider_releases_the_connections_of_finished_tasks(native):
    """A NodeManager's provider outlives thousands of reduce tasks: the sockets and reader threads of a
    task's connections go when the task does, not at provider shutdown."""
    port = _port()
    prov = UdaProvider(transport="tcp", data_port=port, conf={"mapred.uda.provider.bind.address": "127.0.0.1"})
    try:
        job = "job_7_0002"
        maps = datagen.terasort(num_maps=3, reducers=1, rows_per_map=500, seed=79)
        ids = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_{job}_m_{i:06d}_0"
            data, index = encode_partitions(parts, None)
            prov.add_mof_memory(job, mid, data, index)
            ids.append(mid)
        want = sum(len(m[0]) for m in maps)
        rc, out = _task(native, port, job, ids, 0, want)
        assert rc == 0 and out["error"] == "", out
        fds0 = len(os.listdir("/proc/self/fd"))
        for _ in range(12):
            rc, out = _task(native, port, job, ids, 0, want)
            assert rc == 0 and out["error"] == "", out
        # the provider reaps a finished connection when the next one arrives: allow one task's worth
        assert len(os.listdir("/proc/self/fd")) - fds0 <= 8
    finally:
        prov.close()


def _service_provider(tmp_path, port):
    path = str(tmp_path / "merge.sock")
    prov = UdaProvider(transport="tcp", data_port=port, conf={"mapred.uda.provider.bind.address": "127.0.0.1",
                                                              "mapred.uda.gpu.merge.service": path})
    job = "job_8_0001"
    maps = datagen.terasort(num_maps=4, reducers=3, rows_per_map=1500, seed=78)
    ids = []
    for i, parts in enumerate(datagen.streams(maps)):
        mid = f"attempt_{job}_m_{i:06d}_0"
        data, index = encode_partitions(parts, None)
        prov.add_mof_memory(job, mid, data, index)
        ids.append(mid)
    return prov, path, job, maps, ids


@pytest.mark.skipif(not os.access(EXE, os.X_OK), reason="uda_reduce_task not built")
def test_reduce_tasks_hosted_by_the_merge_service(native, tmp_path):
    """mapred.uda.gpu.merge.service: the reduce task processes are thin clients; their NetMergers run in
    the provider's process (commands, configuration pulls, dataFromUda and the stats cross a Unix
    socket). Three tasks at once, each must deliver its partition in order."""
    import concurrent.futures as cf
    port = _port()
    prov, path, job, maps, ids = _service_provider(tmp_path, port)
    try:
        def run(r):
            want = sum(len(m[r]) for m in maps)
            return want, _task(native, port, job, ids, r, want, order=True, extra=["-D", f"mapred.uda.gpu.merge.service={path}"])
        with cf.ThreadPoolExecutor(3) as ex:
            outs = list(ex.map(run, range(3)))
        for want, (rc, out) in outs:
            assert rc == 0 and out["error"] == "", out
            assert out["records"] == want and out["order_errors"] == 0
            assert out["task"].get("merge_service") is True and out["task"]["maps_fetched"] == 4
    finally:
        prov.close()


@pytest.mark.skipif(not os.access(EXE, os.X_OK), reason="uda_reduce_task not built")
def test_merge_service_survives_a_dead_client_and_reports_failures(native, tmp_path):
    """A client killed mid-task leaves the service serving the next task; a task whose FETCH names a map
    the provider does not have fails in its own process (failureInUda), as an in-process task would;
    an unreachable service means the task merges in its own process."""
    port = _port()
    prov, path, job, maps, ids = _service_provider(tmp_path, port)
    try:
        argv = [EXE, "-D", "mapred.uda.transport=tcp", "-D", "mapred.uda.merge.backend=cpu",
                "-D", f"mapred.uda.gpu.merge.service={path}", "--", "-w", "256", "-r", str(port), "-a", "1", "-m",
                "1", "-g", "/tmp", "-s", "1024"]
        init = native.form_cmd(INIT, [str(len(ids)), job, f"attempt_{job}_r_000001_0", "0", str(1 << 20),
                                      str(16 << 10), datagen.TEXT, "null", str(256 << 10), "0", "0"])
        p = subprocess.Popen(argv, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
        p.stdin.write(init + "\n")
        p.stdin.flush()
        import time
        time.sleep(0.5)
        p.kill()
        p.wait()
        want = sum(len(m[1]) for m in maps)
        rc, out = _task(native, port, job, ids, 1, want, order=True, extra=["-D", f"mapred.uda.gpu.merge.service={path}"])
        assert rc == 0 and out["records"] == want and out["task"].get("merge_service") is True, out
        rc, out = _task(native, port, job, ids[:3] + [f"attempt_{job}_m_000099_0"], 2, 1,
                        extra=["-D", f"mapred.uda.gpu.merge.service={path}"])
        assert rc == 1 and out["error"], out
        rc, out = _task(native, port, job, ids, 0, sum(len(m[0]) for m in maps),
                        extra=["-D", f"mapred.uda.gpu.merge.service={tmp_path}/none.sock"])
        assert rc == 0 and "merge_service" not in out["task"], out
    finally:
        prov.close()


@pytest.mark.skipif(not os.access(EXE, os.X_OK), reason="uda_reduce_task not built")
def test_task_fails_cleanly_when_the_merge_service_goes_away(native, tmp_path):
    """The service's process ends while a hosted task waits for its remaining FETCHes: the task
    process reports the failure (failureInUda -> Hadoop's vanilla shuffle) and exits instead of hanging."""
    import time
    port = _port()
    prov, path, job, maps, ids = _service_provider(tmp_path, port)
    try:
        argv = [EXE, "-D", "mapred.uda.transport=tcp", "-D", "mapred.uda.merge.backend=cpu",
                "-D", f"mapred.uda.gpu.merge.service={path}", "--", "-w", "256", "-r", str(port), "-a", "1", "-m",
                "1", "-g", "/tmp", "-s", "1024"]
        init = native.form_cmd(INIT, [str(len(ids)), job, f"attempt_{job}_r_000000_0", "0", str(1 << 20),
                                      str(16 << 10), datagen.TEXT, "null", str(256 << 10), "0", "0"])
        p = subprocess.Popen(argv, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
        p.stdin.write(init + "\n" + native.form_cmd(FETCH, ["127.0.0.1", job, ids[0], "0"]) + "\n")
        p.stdin.flush()
        time.sleep(0.5)
    finally:
        prov.close()  # stops the merge service with the supplier
    out, _ = p.communicate(timeout=60)
    res = json.loads(out.strip().splitlines()[-1])
    assert p.returncode == 1 and "merge service" in res["error"], res
