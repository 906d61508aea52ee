"""Binary distribution layout (tools/package.py): libuda.so finds the node daemon it
starts at <lib>/../bin/uda_mof_supplier (NodeDaemonClient::default_exe), so the package must put it there."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _package_module():
    spec = importlib.util.spec_from_file_location("uda_package", os.path.join(ROOT, "tools", "package.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "uda_amd", "bin", "uda_mof_supplier")), reason="apps not built")
def test_package_puts_the_daemon_next_to_libuda(tmp_path):
    dest = tmp_path / "uda-amd"
    _package_module().stage(str(dest))
    lib = dest / "lib" / "libuda.so"
    assert lib.exists()
    daemon = dest / "lib" / ".." / "bin" / "uda_mof_supplier"
    assert daemon.exists() and os.access(daemon, os.X_OK)
    assert (dest / "bin" / "uda_reduce_task").exists()
    assert (dest / "VERSION").read_text().strip()
