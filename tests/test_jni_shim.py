"""JNI entry points of libuda.so driven by a fake JVM (tests/native/fake_jvm.cc).

The fake JVM plays the Java plugin (UdaBridge.java): JNI_OnLoad, startNative for a MOFSupplier and
a NetMerger, doCommandNative with INIT/FETCH, reduceExitMsgNative, EXIT. Its callbacks check what a
real JVM would enforce: callbacks only on attached threads, dataFromUda handed a direct buffer,
balanced local references, and a bad command raising UdaRuntimeException in the caller.
"""
import json
import os
import shutil
import subprocess

import pytest

from uda_amd.utils import datagen
from uda_amd.utils.ifile import decode_stream
from uda_amd.utils.mof import CODEC_CLASSES, write_mof

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBUDA = os.path.join(ROOT, "uda_amd", "lib", "libuda.so")
EXIT, INIT, FETCH = 0, 7, 4


@pytest.fixture(scope="session")
def fake_jvm(tmp_path_factory, native):  # `native` makes sure the build is present
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path_factory.mktemp("jvm") / "fake_jvm")
    subprocess.run([cxx, "-std=c++17", "-O1", "-pthread", os.path.join(ROOT, "tests", "native", "fake_jvm.cc"),
                    "-o", exe, "-ldl"], check=True)
    return exe


def _manifest(native, path, mofs, maps, job, reduce_id, extra_fetch=(), codec=None, kv_buf=64 << 10, service=None):
    lines = [
        "conf mapred.uda.transport loopback",
        "conf mapred.uda.loopback.host *",
        f"conf mapred.uda.kv.buf.size {kv_buf}",
    ]
    if service:  # the provider hosts the merge service and the NetMerger is its client
        lines.append(f"conf mapred.uda.gpu.merge.service {service}")
        lines.append("loglevel 4")  # info: the start logs where the NetMerger runs
    for a in ["-w", "256", "-r", "9011", "-m", "1", "-g", "/tmp", "-s", "1024"]:
        lines.append(f"parg {a}")
    for a in ["-w", "256", "-r", "9011", "-a", "1", "-m", "1", "-g", "/tmp", "-s", "64"]:
        lines.append(f"carg {a}")
    for mid, (file_out, index) in mofs.items():
        for r, (start, raw, part) in enumerate(index):
            lines.append(f"mof {job} {mid} {r} {start} {raw} {part} {file_out}")
    lines.append("bad 3:this-is-not-a-command")
    params = [str(len(mofs) + len(extra_fetch)), job, f"attempt_{job}_r_{reduce_id:06d}_0", "0", str(64 * 1024),
              str(16 * 1024), datagen.TEXT, CODEC_CLASSES.get(codec, codec) or "null", str(256 * 1024), "0", "0"]
    lines.append("cmd " + native.form_cmd(INIT, params))
    for mid in list(mofs) + list(extra_fetch):
        lines.append("cmd " + native.form_cmd(FETCH, ["localhost", job, mid, str(reduce_id)]))
    lines.append("exit " + native.form_cmd(EXIT, []))
    lines.append(f"out {path}.out")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def _run(fake_jvm, manifest):
    p = subprocess.run([fake_jvm, LIBUDA, manifest], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("codec,service", [(None, False), ("snappy", False), (None, True)])
def test_jni_reduce_through_fake_jvm(native, fake_jvm, tmp_path, codec, service):
    """With the merge service, dataFromUda / fetchOverMessage come from the client's socket threads:
    the shim must attach them like any other native thread."""
    maps = datagen.secondary_sort(num_maps=9, reducers=2, rows_per_map=400, seed=31)
    job = "job_jni_" + (codec or "raw")
    mofs = {}
    for i, parts in enumerate(datagen.streams(maps)):
        mid = f"attempt_{job}_m_{i:06d}_0"
        mofs[mid] = write_mof(str(tmp_path), mid, parts, codec=codec)
    m = str(tmp_path / "manifest.txt")
    _manifest(native, m, mofs, maps, job, 1, codec=codec, service=str(tmp_path / "svc.sock") if service else None)
    st = _run(fake_jvm, m)
    assert st["onload_version"] == 0x00010004
    assert st["start_rc"] == 0 and st["finished"] and st["failures"] == 0
    assert st["bad_cmd_exceptions"] == 1, st
    assert st["unexpected_exceptions"] == 0, st
    assert st["unattached_calls"] == 0 and st["non_direct"] == 0 and st["bad_slot"] == 0
    assert st["live_local_refs"] == 0
    assert st["attaches"] >= 1 and st["detaches"] == st["attaches"]
    assert st["fetch_over"] >= 1 and st["buffers"] >= 2
    assert st["hosted"] == (1 if service else 0), st
    got = decode_stream(open(m + ".out", "rb").read())
    want = sorted((kv for mp in maps for kv in mp[1]), key=datagen.sort_key(datagen.TEXT))
    kf = datagen.sort_key(datagen.TEXT)
    assert [kf(kv) for kv in got] == [kf(kv) for kv in want]
    assert sorted(got) == sorted(want)


def test_jni_missing_mof_calls_failure_once(native, fake_jvm, tmp_path):
    maps = datagen.wordcount(num_maps=2, reducers=1, words_per_map=300)
    job = "job_jni_fail"
    mofs = {}
    for i, parts in enumerate(datagen.streams(maps)):
        mid = f"attempt_{job}_m_{i:06d}_0"
        mofs[mid] = write_mof(str(tmp_path), mid, parts)
    m = str(tmp_path / "manifest.txt")
    _manifest(native, m, mofs, maps, job, 0, extra_fetch=[f"attempt_{job}_m_999999_0"])
    st = _run(fake_jvm, m)
    assert st["failures"] == 1, st
    assert st["unattached_calls"] == 0 and st["live_local_refs"] == 0
