"""CPU tier: the deployment as documented -- a provider front end (the NodeManager's aux service) and
reduce task processes (one per ReduceTask JVM), both with the library's defaults -- and the node daemon
that holds the node's GPU state and hosts the reduce tasks' NetMergers.

* Defaults: no mapred.uda.* key on either side. The reduce task fetches over TCP from the provider
  process (the reference's consumer always builds a network client, src/Merger/reducer.cc:412-437) and
  merges on the CPU here (mapred.uda.merge.backend=auto: no HIP device).
* Node daemon (forced on with mapred.uda.daemon=1, since this machine has no GPU driver): reduce tasks
  with default configuration are hosted by its merge service; a fault injected into one hosted task fails
  that task only (failureInUda exactly once, the others validated); a daemon killed mid-task fails the
  hosted task of that moment while the front end keeps serving byte fetches and restarts the daemon.
* Access: the merge service admits clients by their peer credentials (SO_PEERCRED) against
  mapred.uda.gpu.merge.service.users.

Reference: src/UdaBridge.cc:506-530 (a native failure falls back for that reducer only),
plugins/shared/.../UdaShuffleConsumerPluginShared.java:205-232, src/MOFServer/MOFSupplierMain.cc:87-143."""
import json
import os
import shutil
import signal
import socket
import subprocess
import time

import pytest

from uda_amd.bridge import FETCH, INIT
from uda_amd.utils import datagen
from uda_amd.utils.mof import write_mof

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUP = os.path.join(ROOT, "uda_amd", "bin", "uda_mof_supplier")
EXE = os.path.join(ROOT, "uda_amd", "bin", "uda_reduce_task")
pytestmark = pytest.mark.skipif(not (os.access(SUP, os.X_OK) and os.access(EXE, os.X_OK)), reason="apps not built")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class FrontEnd:
    """uda_mof_supplier mode=frontend: uda_start(provider) with getPathUda over Hadoop-layout MOFs."""

    def __init__(self, mof_dir, port, conf=None, pass_fds=()):
        argv = [SUP, "mode=frontend", f"mof_dir={mof_dir}", f"port={port}"]
        for k, v in (conf or {}).items():
            argv.append(f"-D{k}={v}")
        self.p = subprocess.Popen(argv, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, cwd=ROOT,
                                  pass_fds=pass_fds)
        line = self.p.stdout.readline()
        assert line, f"front end exited rc={self.p.poll()}"
        self.info = json.loads(line)
        self.port = port

    def stats(self):
        self.p.stdin.write("stats\n")
        self.p.stdin.flush()
        return json.loads(self.p.stdout.readline())

    def close(self):
        if self.p.poll() is None:
            try:
                self.p.stdin.write("exit\n")
                self.p.stdin.flush()
                self.p.wait(60)
            except (OSError, subprocess.TimeoutExpired):
                self.p.kill()
                self.p.wait()


def _job(tmp_path, job, maps=4, reducers=3, rows=1200, seed=5):
    d = tmp_path / "mofs"
    data = datagen.terasort(num_maps=maps, reducers=reducers, rows_per_map=rows, seed=seed)
    ids = []
    for i, parts in enumerate(datagen.streams(data)):
        mid = f"attempt_{job}_m_{i:06d}_0"
        write_mof(str(d), mid, parts)
        ids.append(mid)
    return str(d), data, ids


def _cmds(native, job, ids, r, local_dirs=()):
    init = native.form_cmd(INIT, [str(len(ids)), job, f"attempt_{job}_r_{r:06d}_0", "0", str(1 << 20),
                                  str(16 << 10), datagen.TEXT, "null", str(256 << 10), "0",
                                  str(len(local_dirs)), *local_dirs])
    return [init] + [native.form_cmd(FETCH, ["127.0.0.1", job, m, str(r)]) for m in ids]


def _task_argv(port, expect, conf=(), exe=EXE):
    argv = [exe]
    for kv in conf:
        argv += ["-D", kv]
    return argv + ["--expect", str(expect), "--check-order", "--", "-w", "256", "-r", str(port), "-a", "1",
                   "-m", "1", "-g", "/tmp", "-s", "1024"]


def _run_task(native, port, job, ids, r, expect, conf=(), exe=EXE, local_dirs=(), **popen):
    p = subprocess.run(_task_argv(port, expect, conf, exe),
                       input="\n".join(_cmds(native, job, ids, r, local_dirs)) + "\n",
                       capture_output=True, text=True, timeout=120, **popen)
    lines = p.stdout.strip().splitlines()
    assert lines, f"no output, rc={p.returncode}, stderr={p.stderr[-2000:]}"
    return p.returncode, json.loads(lines[-1])


def _want(data, r):
    return sum(len(m[r]) for m in data)


def test_default_configuration_fetches_across_processes(native, tmp_path):
    """zero mapred.uda.* keys in the provider process and in the reduce task process.
    Before: loopback transport by default ("no loopback provider for host") and a CPU-only default."""
    job = "job_50_0001"
    mof_dir, data, ids = _job(tmp_path, job)
    port = _port()
    fe = FrontEnd(mof_dir, port)
    try:
        for r in range(3):
            rc, out = _run_task(native, port, job, ids, r, _want(data, r))
            assert rc == 0 and out["error"] == "", out
            assert out["records"] == _want(data, r) and out["order_errors"] == 0
            t = out["task"]
            assert t["maps_fetched"] == 4 and t["bytes_fetched"] > 0, t
            assert t["backend"] == ("gpu" if native.device_count() > 0 else "cpu"), t  # merge.backend=auto
        st = fe.stats()
        assert st["port"] == port and st["requests"] >= 12, st
    finally:
        fe.close()


def test_daemon_does_not_inherit_front_end_descriptors(tmp_path):
    """A NodeManager JVM holds descriptors without close-on-exec (listening sockets, logs); the daemon it
    starts closes every inherited descriptor but its control socket, so it never keeps the NodeManager's
    port or files open."""
    mof_dir, _, _ = _job(tmp_path, "job_fds")
    marker = tmp_path / "nodemanager-held.log"
    fd = os.open(str(marker), os.O_WRONLY | os.O_CREAT, 0o644)  # inheritable (no O_CLOEXEC in the child)
    fe = None
    try:
        fe = FrontEnd(mof_dir, _port(), {"mapred.uda.daemon": "1"}, pass_fds=(fd,))
        dpid = fe.info["provider"]["hbm_store"]["daemon"]["pid"]
        fepid = fe.p.pid

        def targets(pid):
            out = set()
            for e in os.listdir(f"/proc/{pid}/fd"):
                try:
                    out.add(os.readlink(f"/proc/{pid}/fd/{e}"))
                except OSError:
                    pass
            return out

        assert str(marker) in targets(fepid)  # the front end (the "JVM") holds it
        assert str(marker) not in targets(dpid), targets(dpid)
    finally:
        os.close(fd)
        if fe is not None:
            fe.close()


def test_daemon_and_front_end_descriptor_tables_are_grown_up_front(tmp_path):
    """A multi-threaded process's descriptor table grows by doubling, each doubling waiting for an RCU grace
    period while every thread that opens a descriptor waits with it (the daemon's first-wave freeze,
    profiles/r6/r7_first_wave_stall.md): the daemon and the front end grow theirs before their threads
    start (FDSize in /proc/<pid>/status), up to the descriptor limit."""
    import resource

    mof_dir, _, _ = _job(tmp_path, "job_fdsize")
    fe = FrontEnd(mof_dir, _port(), {"mapred.uda.daemon": "1"})
    try:
        want = min(resource.getrlimit(resource.RLIMIT_NOFILE)[1], 1 << 17)
        for pid in (fe.p.pid, fe.info["provider"]["hbm_store"]["daemon"]["pid"]):
            with open(f"/proc/{pid}/status") as f:
                size = int(next(l for l in f if l.startswith("FDSize:")).split()[1])
            assert size >= want, (pid, size, want)
    finally:
        fe.close()


def test_daemon_starts_with_its_allocator_tunables(tmp_path, monkeypatch):
    """The daemon is spawned with glibc tunables that keep a wave of task starts from queueing on the
    address-space lock (cached thread stacks, few arenas made writable whole); a GLIBC_TUNABLES of the
    front end's environment is kept, with the daemon's settings after it."""
    mof_dir, _, _ = _job(tmp_path, "job_tun")
    monkeypatch.setenv("GLIBC_TUNABLES", "glibc.malloc.tcache_count=5")
    fe = FrontEnd(mof_dir, _port(), {"mapred.uda.daemon": "1"})
    try:
        # glibc's own view in the daemon (/proc/<pid>/environ shows the string as glibc's parse cut it)
        tun = fe.stats()["hbm_store"]["glibc_tunables"]
        assert tun.startswith("glibc.malloc.tcache_count=5:"), tun
        for want in ("glibc.pthread.stack_cache_size=1073741824", "glibc.malloc.arena_max=8", "glibc.malloc.top_pad=67108864"):
            assert want in tun, tun
    finally:
        fe.close()


def _daemon_front(tmp_path, job, conf=None, **kw):
    mof_dir, data, ids = _job(tmp_path, job, **kw)
    port = _port()
    c = {"mapred.uda.daemon": "1"}  # no GPU driver here: force the daemon on (a GPU node starts it by default)
    c.update(conf or {})
    fe = FrontEnd(mof_dir, port, c)
    d = fe.info["provider"]["hbm_store"]["daemon"]
    assert d["ready"] is True and d["pid"] > 0 and d["service"] == f"@uda-merge-{port}", fe.info
    # no GPU to prewarm for: the daemon reports its first-wave prewarm as done (what a bench waits for)
    pw = fe.stats()["hbm_store"].get("prewarm")
    assert pw is not None and pw["done"] is True, pw
    return fe, data, ids, port


def test_daemon_hosts_default_tasks_and_contains_a_task_fault(native, tmp_path):
    """Four reduce task processes with default configuration are hosted by the node daemon's merge service;
    one of them carries an injected fault (its own mapred.uda.fault.inject, applied on its merge thread
    only): exactly that task fails (failureInUda once), the other three deliver validated streams, and the
    daemon keeps running."""
    import concurrent.futures as cf
    job = "job_50_0002"
    fe, data, ids, port = _daemon_front(tmp_path, job, reducers=4)
    try:
        pid0 = fe.stats()["hbm_store"]["daemon"]["pid"]

        def run(r):
            conf = ["mapred.uda.fault.inject=FETCH=2"] if r == 2 else []
            return r, _run_task(native, port, job, ids, r, _want(data, r), conf)

        with cf.ThreadPoolExecutor(4) as ex:
            outs = dict(ex.map(run, range(4)))
        for r, (rc, out) in outs.items():
            if r == 2:
                assert rc == 1 and "injected fetch failure" in out["error"], out
            else:
                assert rc == 0 and out["error"] == "" and out["records"] == _want(data, r), out
                assert out["task"].get("merge_service") is True, out["task"]
        st = fe.stats()
        d = st["hbm_store"]["daemon"]
        assert d["pid"] == pid0 and d["ready"] is True and d["restarts"] == 0, d
        ms = st["hbm_store"]["merge_service"]
        assert ms["sessions"] >= 4 and ms["refused"] == 0, ms
    finally:
        fe.close()


def test_daemon_death_fails_hosted_tasks_only_and_is_restarted(native, tmp_path):
    """The daemon dies (SIGKILL, as after a GPU fault) while a hosted task waits for its FETCHes: that task
    reports the failure and exits; the front end keeps answering byte fetches (a task merging in its own
    process is served) and restarts the daemon, whose service hosts the next default task."""
    job = "job_50_0003"
    fe, data, ids, port = _daemon_front(tmp_path, job)
    try:
        pid0 = fe.stats()["hbm_store"]["daemon"]["pid"]
        cmds = _cmds(native, job, ids, 0)
        p = subprocess.Popen(_task_argv(port, _want(data, 0)), stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                             stderr=subprocess.DEVNULL, text=True)
        p.stdin.write(cmds[0] + "\n" + cmds[1] + "\n")  # INIT + one FETCH; the rest never comes
        p.stdin.flush()
        time.sleep(1.0)
        os.kill(pid0, signal.SIGKILL)
        out, _ = p.communicate(timeout=60)
        res = json.loads(out.strip().splitlines()[-1])
        assert p.returncode == 1 and "merge service" in res["error"], res
        # byte fetches from the front end go on while the daemon is down or restarting
        rc, out = _run_task(native, port, job, ids, 1, _want(data, 1), ["mapred.uda.gpu.merge.service=off"])
        assert rc == 0 and out["records"] == _want(data, 1) and "merge_service" not in out["task"], out
        t0 = time.time()
        while time.time() - t0 < 30:
            d = fe.stats()["hbm_store"]["daemon"]
            if d["ready"]:
                break
            time.sleep(0.2)
        assert d["ready"] is True and d["restarts"] == 1 and d["pid"] not in (0, pid0), d
        rc, out = _run_task(native, port, job, ids, 2, _want(data, 2))
        assert rc == 0 and out["task"].get("merge_service") is True, out
        assert fe.p.poll() is None  # the front end (the NodeManager) never went down
    finally:
        fe.close()


@pytest.fixture
def request_cleanup():
    dirs = []
    yield dirs
    for d in dirs:
        shutil.rmtree(d, ignore_errors=True)


def test_merge_service_user_rule(native):
    me = os.getuid()
    assert native.merge_service_user_allowed("", me)  # the service's own user always may
    assert native.merge_service_user_allowed("*", 4242)
    assert native.merge_service_user_allowed("root,4242", 4242)
    assert native.merge_service_user_allowed(" nobody ", 65534)
    assert not native.merge_service_user_allowed("root,4243", 4242)
    assert not native.merge_service_user_allowed("", 4242)
    assert native.merge_service_default_path(9011) == "@uda-merge-9011"


@pytest.mark.skipif(os.geteuid() != 0, reason="needs root to run a task process as another user")
def test_merge_service_admits_by_peer_credentials(native, request_cleanup):
    """A task process of a user outside mapred.uda.gpu.merge.service.users is refused (and merges in its
    own process); listed, it is hosted. By default (no key) only the service's own user is hosted."""
    # the task binary, its library and the MOFs where user nobody can read them (pytest's tmp_path is
    # private to root)
    import pathlib
    import tempfile
    tmp_path = pathlib.Path(tempfile.mkdtemp(prefix="uda-peercred-"))
    request_cleanup.append(tmp_path)
    app = tmp_path / "app"
    (app / "bin").mkdir(parents=True)
    (app / "lib").mkdir()
    shutil.copy2(EXE, app / "bin" / "uda_reduce_task")
    shutil.copy2(os.path.join(ROOT, "uda_amd", "lib", "libuda.so"), app / "lib" / "libuda.so")
    for x in (tmp_path, app, app / "bin", app / "lib"):
        os.chmod(x, 0o755)
    exe = str(app / "bin" / "uda_reduce_task")

    def as_nobody():
        os.setgid(65534)
        os.setuid(65534)

    for k, (users, hosted) in enumerate(((None, False), ("root", False), ("root,nobody", True))):
        job = f"job_50_00{4 + k}"
        sub = tmp_path / job
        sub.mkdir()
        os.chmod(sub, 0o755)
        conf = {} if users is None else {"mapred.uda.gpu.merge.service.users": users}
        fe, data, ids, port = _daemon_front(sub, job, conf)
        try:
            os.chmod(sub / "mofs", 0o755)
            rc, out = _run_task(native, port, job, ids, 0, _want(data, 0), exe=exe, preexec_fn=as_nobody, cwd="/tmp")
            assert rc == 0 and out["records"] == _want(data, 0), out
            assert (out["task"].get("merge_service") is True) == hosted, out["task"]
            ms = fe.stats()["hbm_store"]["merge_service"]
            assert (ms["refused"] == 0) == hosted, ms
        finally:
            fe.close()


def _nobody_app(tmp_path):
    """The task binary and its library where user nobody can run them."""
    app = tmp_path / "app"
    (app / "bin").mkdir(parents=True)
    (app / "lib").mkdir()
    shutil.copy2(EXE, app / "bin" / "uda_reduce_task")
    shutil.copy2(os.path.join(ROOT, "uda_amd", "lib", "libuda.so"), app / "lib" / "libuda.so")
    for x in (tmp_path, app, app / "bin", app / "lib"):
        os.chmod(x, 0o755)
    return str(app / "bin" / "uda_reduce_task")


@pytest.mark.skipif(os.geteuid() != 0, reason="needs root to run a task process as another user")
def test_confined_hosted_task_keeps_to_node_local_dirs(native, request_cleanup):
    """A task the service hosts for another user: with local dirs inside the node's own
    (mapred.uda.gpu.merge.service.local.dirs) it is hosted; with a local dir elsewhere the service refuses
    its files and the task merges in its own process (as that user), and nothing of it lands in the
    service's name in the foreign dir; a task id naming a path is refused the same way."""
    import pathlib
    import tempfile
    tmp_path = pathlib.Path(tempfile.mkdtemp(prefix="uda-confine-"))
    request_cleanup.append(tmp_path)
    exe = _nobody_app(tmp_path)
    node_dir = tmp_path / "nm-local"
    elsewhere = tmp_path / "elsewhere"
    for d in (node_dir, elsewhere):
        d.mkdir()
        os.chown(d, 65534, 65534)

    def as_nobody():
        os.setgid(65534)
        os.setuid(65534)

    job = "job_50_0020"
    sub = tmp_path / job
    sub.mkdir()
    os.chmod(sub, 0o755)
    fe, data, ids, port = _daemon_front(sub, job, {"mapred.uda.gpu.merge.service.users": "nobody",
                                                   "mapred.uda.gpu.merge.service.local.dirs": str(node_dir)})
    try:
        os.chmod(sub / "mofs", 0o755)
        for r, dirs, hosted in ((0, (str(node_dir),), True), (1, (str(elsewhere),), False)):
            rc, out = _run_task(native, port, job, ids, r, _want(data, r), exe=exe, local_dirs=dirs,
                                preexec_fn=as_nobody, cwd="/tmp")
            assert rc == 0 and out["records"] == _want(data, r), out
            assert (out["task"].get("merge_service") is True) == hosted, (dirs, out["task"])
        for f in elsewhere.iterdir():  # whatever the in-process task left belongs to its own user
            assert f.lstat().st_uid == 65534, f
    finally:
        fe.close()


def test_client_refuses_a_service_of_an_untrusted_user(native, request_cleanup):
    """The abstract socket name can be bound by anyone first; the client checks the peer's uid before it
    sends its HELLO: a service run by an untrusted uid is not used and the task merges
    in its own process."""
    if os.geteuid() != 0:
        pytest.skip("needs root to run the service as another user")
    import pathlib
    import tempfile
    tmp_path = pathlib.Path(tempfile.mkdtemp(prefix="uda-squat-"))
    request_cleanup.append(tmp_path)
    job = "job_50_0021"
    mof_dir, data, ids = _job(tmp_path, job)
    port = _port()
    fe = FrontEnd(mof_dir, port)  # provider without a daemon: serves bytes
    squat = None
    try:
        # a process of user nobody squats the service name of this port
        code = ("import socket,os,time\n"
                "os.setgid(65534); os.setuid(65534)\n"
                "s=socket.socket(socket.AF_UNIX); s.bind('\\0uda-merge-%d'); s.listen(8)\n"
                "print('up', flush=True)\n"
                "c,_=s.accept(); time.sleep(30)\n" % port)
        squat = subprocess.Popen(["python3", "-c", code], stdout=subprocess.PIPE, text=True)
        assert squat.stdout.readline().strip() == "up"
        rc, out = _run_task(native, port, job, ids, 0, _want(data, 0))
        assert rc == 0 and out["records"] == _want(data, 0), out
        assert "merge_service" not in out["task"], out["task"]
    finally:
        if squat is not None:
            squat.kill()
            squat.wait()
        fe.close()


def test_per_gpu_daemons_contain_a_daemon_death(native, tmp_path):
    """one node daemon per GPU (forced to 2 here, no GPU on this machine). The front end
    routes each reduce task's connections to the daemon with the fewest live sessions: task 0 lands on
    daemon 0, task 1 on daemon 1. Killing daemon 1 mid-task (as a fault on its GPU would) fails task 1 only;
    task 0, hosted by daemon 0, delivers its validated stream; daemon 1 is restarted, daemon 0 never was."""
    job = "job_50_0030"
    fe, data, ids, port = _daemon_front(tmp_path, job, {"mapred.uda.daemon.count": "2"}, reducers=3)
    procs = []
    try:
        def daemons():
            return fe.stats()["hbm_store"]["daemons"]

        def wait_for(pred, what, timeout=30):
            t0 = time.time()
            while time.time() - t0 < timeout:
                ds = daemons()
                if pred(ds):
                    return ds
                time.sleep(0.1)
            raise AssertionError(f"timed out waiting for {what}: {daemons()}")

        ds = wait_for(lambda d: len(d) == 2 and all(x["ready"] for x in d), "two ready daemons")
        assert [d["device"] for d in ds] == [0, 1] and ds[0]["pid"] != ds[1]["pid"], ds
        pid0, pid1 = ds[0]["pid"], ds[1]["pid"]
        cmds = [_cmds(native, job, ids, r) for r in range(2)]
        for r in range(2):  # INIT + one FETCH each; the rest of task 0's FETCHes come after the kill
            p = subprocess.Popen(_task_argv(port, _want(data, r)), stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                 stderr=subprocess.DEVNULL, text=True)
            p.stdin.write(cmds[r][0] + "\n" + cmds[r][1] + "\n")
            p.stdin.flush()
            procs.append(p)
            wait_for(lambda d, r=r: d[r]["live_sessions"] == 1, f"task {r} hosted by daemon {r}")
        os.kill(pid1, signal.SIGKILL)
        out1, _ = procs[1].communicate(timeout=60)
        res1 = json.loads(out1.strip().splitlines()[-1])
        assert procs[1].returncode == 1 and "merge service" in res1["error"], res1
        procs[0].stdin.write("\n".join(cmds[0][2:]) + "\n")
        out0, _ = procs[0].communicate(timeout=120)
        res0 = json.loads(out0.strip().splitlines()[-1])
        assert procs[0].returncode == 0 and res0["error"] == "" and res0["records"] == _want(data, 0), res0
        assert res0["task"].get("merge_service") is True, res0["task"]
        ds = wait_for(lambda d: d[1]["ready"] and d[1]["restarts"] == 1, "daemon 1 restarted")
        assert ds[0]["pid"] == pid0 and ds[0]["restarts"] == 0, ds
        assert ds[1]["pid"] not in (0, pid1), ds
        rc, out = _run_task(native, port, job, ids, 2, _want(data, 2))  # the node keeps hosting tasks
        assert rc == 0 and out["task"].get("merge_service") is True, out
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        fe.close()
