"""CPU tier: the executables name a fatal signal and print a backtrace before they die of it.

A provider front end or node daemon that dies of a signal otherwise leaves only "connection lost" at its
peers (the r6 node-files run with a store smaller than the map outputs).
"""
import os
import signal
import socket
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUP = os.path.join(ROOT, "uda_amd", "bin", "uda_mof_supplier")


@pytest.mark.parametrize("sig", [signal.SIGSEGV, signal.SIGBUS])
def test_front_end_reports_a_fatal_signal(tmp_path, sig):
    if not os.access(SUP, os.X_OK):
        pytest.skip("uda_mof_supplier not built")
    mofs = tmp_path / "mofs"
    mofs.mkdir()
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, UDA_DAEMON_LOG=str(tmp_path / "daemon.log"))
    p = subprocess.Popen([SUP, "mode=frontend", f"mof_dir={mofs}", f"port={port}", "-Dmapred.uda.daemon=off"],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    try:
        assert p.stdout.readline().strip().startswith("{")  # up: its first JSON line
        time.sleep(0.2)
        p.send_signal(sig)
        _, err = p.communicate(timeout=30)
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
    assert p.returncode == -sig  # still dies of the signal (a core dump / the parent's view unchanged)
    assert f"uda_mof_supplier pid {p.pid}: fatal signal {int(sig)}" in err
    assert "uda_mof_supplier" in err.split("fatal signal", 1)[1] or "libuda" in err  # backtrace frames
