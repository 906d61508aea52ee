"""Unit tests for the native common layer: VInt codec, command protocol, options, comparators."""
import random

import pytest

from uda_amd.utils import ifile


VINT_CASES = [0, 1, -1, 127, 128, -112, -113, 255, 256, -256, 65535, 65536, 2**31 - 1, -2**31,
              2**40, -2**40, 2**63 - 1, -2**63]


@pytest.mark.parametrize("v", VINT_CASES)
def test_vint_matches_hadoop_writable_utils(native, v):
    enc = native.vint_encode(v)
    assert enc == ifile.vint_encode(v)
    assert native.vint_decode(enc) == (v, len(enc))
    assert native.vint_size(v) == len(enc)
    first = enc[0] - 256 if enc[0] > 127 else enc[0]
    assert native.vint_decode_size(first) == len(enc)
    assert ifile.vint_decode(enc) == (v, len(enc))


def test_vint_random_roundtrip(native):
    rng = random.Random(7)
    for _ in range(2000):
        v = rng.randint(-2**63, 2**63 - 1) >> rng.randint(0, 63)
        assert native.vint_decode(native.vint_encode(v)) == (v, native.vint_size(v))


def test_vint_truncated(native):
    assert native.vint_decode(b"\x8e")[1] == 0  # length byte promises 2 more bytes


def form_cmd_java(cmd, params):
    # UdaCmd.formCmd (UdaPlugin.java:577-586)
    ret = f"{len(params) + 1}:{cmd}"
    for p in params:
        ret += ":" + p
    return ret


@pytest.mark.parametrize("params", [[], ["a"], ["host1", "job_1", "attempt_1_m_000001_0", "3"],
                                    ["x", "/path/with:colon"]])
def test_command_format_parity(native, params):
    assert native.form_cmd(4, params) == form_cmd_java(4, params)
    count, header, got = native.parse_cmd(form_cmd_java(4, params))
    assert (count, header) == (len(params) + 1, 4)
    assert got == params


def test_command_edge_cases(native):
    assert native.parse_cmd("") == (1, 0, [])          # empty == EXIT
    assert native.parse_cmd("1:0") == (1, 0, [])
    with pytest.raises(ValueError):
        native.parse_cmd("garbage")
    with pytest.raises(ValueError):
        native.parse_cmd("4:7:a")                        # declares 3 params, carries 1


def test_init_command_params_roundtrip(native):
    params = ["12", "job_201208301702_0002", "attempt_201208301702_0002_r_000002_0", "0",
              str(1024 * 1024), str(16 * 1024), "org.apache.hadoop.io.Text", "null", str(256 * 1024),
              str(1 << 30), "2", "/data1/mapred/local", "/data2/mapred/local"]
    count, header, got = native.parse_cmd(native.form_cmd(7, params))
    assert header == 7 and got == params


def test_options_parser(native):
    d = native.parse_options(["-w", "128", "-r", "9100", "-a", "2", "-m", "1", "-g", "/tmp/logs", "-s", "1023"])
    assert d["wqes_per_conn"] == 128 and d["data_port"] == 9100 and d["online"] == 2
    assert d["log_dir"] == "/tmp/logs"
    assert d["buf_size"] == 1023 * 1024 - (1023 * 1024) % 4096   # KB -> bytes, 4 KiB aligned


TEXT, INT, BYTES = "org.apache.hadoop.io.Text", "org.apache.hadoop.io.IntWritable", "org.apache.hadoop.io.BytesWritable"


def test_key_classes(native):
    assert native.key_kind(TEXT) == 0
    for c in ("BooleanWritable", "ByteWritable", "ShortWritable", "IntWritable", "LongWritable"):
        assert native.key_kind("org.apache.hadoop.io." + c) == 1
    assert native.key_kind(BYTES) == 2
    assert native.key_kind("org.apache.hadoop.hbase.io.ImmutableBytesWritable") == 2
    assert native.key_kind("org.apache.hadoop.io.DoubleWritable") == -1


def sign(x):
    return (x > 0) - (x < 0)


def test_text_comparator_skips_vint_prefix(native):
    rng = random.Random(3)
    for _ in range(500):
        a = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 300)))
        b = a[:rng.randint(0, len(a))] + bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 3)))
        got = sign(native.key_compare(0, ifile.text(a), ifile.text(b)))
        assert got == sign((a > b) - (a < b))


def test_raw_and_bytes_comparators(native):
    assert native.key_compare(1, (5).to_bytes(4, "big"), (7).to_bytes(4, "big")) < 0
    assert native.key_compare(1, b"\x00\x01", b"\x00\x01\x00") < 0  # tie on prefix -> shorter first
    bw = lambda s: len(s).to_bytes(4, "big") + s  # noqa: E731
    assert native.key_compare(2, bw(b"abc"), bw(b"abd")) < 0
    assert native.key_compare(2, bw(b"b"), bw(b"abc")) > 0   # length prefix is skipped, not compared


def test_parse_cmd_rejects_garbled_headers(native):
    import pytest as _pytest
    for bad in ["3:this-is-not-a-command", "x:7:a:b", "2:12:p", "2:-1:p", ":7", "nocolon"]:
        with _pytest.raises(ValueError):
            native.parse_cmd(bad)
    assert native.parse_cmd("2:4:p")[1] == 4


def test_topology_plan_and_peer_order():
    from uda_amd.utils import topology
    t = topology.topology()
    assert t["devices"] >= 0 and isinstance(t["links"], list)
    for w in (1, 2, 4, 8):
        for r in range(w):
            order = topology.peer_order(r, w)
            assert sorted(s for s, _ in order) == sorted(set(range(w)) - {r})
            assert sorted(f for _, f in order) == sorted(set(range(w)) - {r})
    p = topology.shuffle_plan(8, 130 << 30)
    assert p["rounds"] >= 1 and p["bytes_per_round"] * p["rounds"] <= 130 << 30


def test_ipc_safe_bytes_avoids_the_hanging_size_range(native):
    """Blocks mapped by another process over hipIpc must not have size % 2^32 in [2^31, 2^32): that
    range hangs the importer on this ROCm (tools/ipc_size_probe.py). Sizes outside it are unchanged."""
    G = 1 << 30
    for size in [1, 1 << 20, G, 2 * G - 1, 4 * G, 4 * G + G, 130 * 10**9]:
        if (size % (4 * G)) < 2 * G:
            assert native.ipc_safe_bytes(size) == size
    for size in [2 * G, 2 * G + 1, 3 * G, 4 * G - 1, 8 * 10**9, 6 * G + 12345]:
        padded = native.ipc_safe_bytes(size)
        assert padded >= size
        assert padded % (4 * G) < 2 * G
        assert padded - size <= 2 * G + (64 << 20)


def test_device_descriptor_identity(native):
    """A descriptor carries the provider's node identity (hostname + boot id): one from another node
    or container is never mapped (the reducer fetches bytes instead); a same-process descriptor
    resolves to its address; a descriptor without an IPC handle from another process is refused."""
    import os
    me = native.node_id()
    assert len(me) == 16 and me == native.node_id()
    d = native.descriptor_make(0, 0x7F0000001000, "-", 0x7F0000000000)
    f = d.split("@")
    assert f[0] == "hbm" and f[1] == me and int(f[3]) == os.getpid() and f[6] == str(0x1000)
    addr, why = native.descriptor_resolve(d, 0)  # same process, same device: the address itself
    assert addr == 0x7F0000001000, why
    forged = "@".join([f[0], "0123456789abcdef"] + f[2:])  # same pid/address, other node
    addr, why = native.descriptor_resolve(forged, 0)
    assert addr is None and "another node" in why
    other_pid = "@".join(f[:3] + [str(os.getpid() + 1)] + f[4:])
    addr, why = native.descriptor_resolve(other_pid, 0)
    assert addr is None and "not IPC-shareable" in why
    for bad in ("hbm@1@2", "hbm@" + me + "@0@1@zz@-", "mem:job/map"):
        assert native.descriptor_resolve(bad, 0)[0] is None


def test_ipc_export_size_rule(native):
    for size in (1 << 20, (1 << 31) - 1, 1 << 32, (1 << 32) + (1 << 30), 5 << 30):
        assert native.ipc_size_ok(size), size
    for size in (1 << 31, 3 << 30, (1 << 32) - 1, (6 << 30) + 1):
        assert not native.ipc_size_ok(size), size
        assert native.ipc_size_ok(native.ipc_safe_bytes(size))


def test_buffer_ends_with_eof_walks_the_framing():
    """The keep_records=False consumer finishes on the EOF marker, found by walking the VInt framing:
    a record whose value ends in 0xFF 0xFF must not pass for the marker (it once ended a 2 GB task
    early, 582 MB in)."""
    from uda_amd import native
    from uda_amd.utils.ifile import encode_record, encode_stream, text
    n = native()
    tricky = encode_record(text(b"k1"), b"abc\xff\xff") + encode_record(text(b"k2"), b"\x00\xff\xff")
    assert tricky.endswith(b"\xff\xff")
    assert n.buffer_ends_with_eof(tricky) == 0
    assert n.buffer_ends_with_eof(tricky + b"\xff\xff") == 1
    assert n.buffer_ends_with_eof(b"\xff\xff") == 1
    assert n.buffer_ends_with_eof(encode_stream([(text(b"a"), b"\xff\xff")])) == 1
    assert n.buffer_ends_with_eof(tricky[:-1]) == -1  # a cut record is broken framing
