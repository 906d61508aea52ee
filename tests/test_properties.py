"""Property tests (Hypothesis): the merge engines against Python's sort on arbitrary run sets
(empty runs, single records, duplicate keys, keys that share long prefixes), and the codecs /
framing / VInt / command layers on arbitrary inputs. SURVEY.md §7.4 "Property"."""
import struct

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from uda_amd import ops
from uda_amd.utils import datagen
from uda_amd.utils.ifile import EOF_MARKER, J2CQueueReader, decode_stream, encode_stream, text

SETTINGS = settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])

_alphabet = st.sampled_from([b"a", b"b", b"ab", b"\x00", b"\xff", b"zzzzzzzz"])
_text_key = st.lists(_alphabet, max_size=8).map(lambda parts: text(b"".join(parts)))
_int_key = st.integers(-2**31, 2**31 - 1).map(lambda v: struct.pack(">i", v))
_bytes_key = st.binary(max_size=12).map(lambda b: len(b).to_bytes(4, "big") + b)
KEYS = {datagen.TEXT: _text_key, datagen.INT: _int_key, datagen.BYTES: _bytes_key}


def _runs(key_class):
    rec = st.tuples(KEYS[key_class], st.binary(max_size=10))
    kf = datagen.sort_key(key_class)
    run = st.lists(rec, max_size=30).map(lambda rs: sorted(rs, key=kf))
    return st.lists(run, min_size=0, max_size=7)


def _stable_expected(runs, key_class):
    kf = datagen.sort_key(key_class)
    flat = [kv for r in runs for kv in r]  # run order, then position: the engines' tie order
    return sorted(flat, key=kf)


@pytest.mark.parametrize("key_class", [datagen.TEXT, datagen.INT, datagen.BYTES])
def test_cpu_merge_equals_sorted(native, key_class):
    @SETTINGS
    @given(runs=_runs(key_class), buf=st.integers(64, 4096))
    def check(runs, buf):
        streams = [encode_stream(r) for r in runs]
        max_rec = max((len(encode_stream([kv], eof=False)) for r in runs for kv in r), default=0)
        buf = max(buf, max_rec + 2)
        out, lens = native.cpu_merge(streams, key_class, buf)
        assert all(n <= buf for n in lens) and out.endswith(EOF_MARKER)
        got = decode_stream(out)
        assert got == _stable_expected(runs, key_class)
        # the buffers are exactly what J2CQueue accepts: whole records, EOF in the last one
        reader = J2CQueueReader(max_len=buf)
        pos = 0
        for n in lens:
            reader.feed(out[pos:pos + n])
            pos += n
        assert reader.eof and reader.records == got

    check()


@pytest.mark.gpu
@pytest.mark.parametrize("key_class", [datagen.TEXT, datagen.INT, datagen.BYTES])
def test_gpu_merge_equals_cpu_merge(require_gpu, key_class):
    @settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])
    @given(runs=_runs(key_class))
    def check(runs):
        streams = [encode_stream(r) for r in runs]
        g, cuts = ops.merge_runs(streams, key_class, "gpu", kv_buf=1024)
        c, _ = ops.merge_runs(streams, key_class, "cpu", kv_buf=1024)
        assert g == c
        assert decode_stream(g + EOF_MARKER) == _stable_expected(runs, key_class)  # merge_runs: records only

    check()


@SETTINGS
@given(v=st.integers(-2**63, 2**63 - 1))
def test_vint_roundtrip_property(native, v):
    enc = native.vint_encode(v)
    assert native.vint_decode(enc) == (v, len(enc))
    assert native.vint_size(v) == len(enc) <= 9


@SETTINGS
@given(data=st.binary(max_size=20000) | st.lists(st.sampled_from([b"ab", b"abc", b"\x00" * 7, b"xyz!"]),
                                                 max_size=3000).map(b"".join),
       block=st.integers(1, 70000), feed=st.integers(1, 9000), codec=st.sampled_from([1, 2]))
def test_block_codecs_roundtrip_any_split(native, data, block, feed, codec):
    framed = native.block_compress(codec, data, block)
    assert native.block_decompress(codec, framed, feed) == data


@SETTINGS
@given(params=st.lists(st.text(alphabet="abcdefghij_0123456789./", min_size=0, max_size=12), max_size=8),
       cmd=st.integers(0, 9))
def test_command_roundtrip_property(native, params, cmd):
    s = native.form_cmd(cmd, params)
    count, header, got = native.parse_cmd(s)
    assert (count, header, got) == (len(params) + 1, cmd, params)
