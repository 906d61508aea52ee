"""Native J2C consumer (the stand-in for the Java reducer's J2CQueue): every buffer is copied into a
KVBuf and walked by its VInt lengths; framing errors, data after EOF and key order are detected."""
import os

import pytest

from uda_amd import native
from uda_amd.utils.ifile import encode_stream, text

EOF_MARK = b"\xff\xff"


def _tera(n, seed=1):
    rnd = __import__("random").Random(seed)
    keys = sorted(bytes(rnd.getrandbits(8) for _ in range(10)) for _ in range(n))
    return encode_stream([(text(k), text(b"V" * 90)) for k in keys])


def test_counts_records_and_eof():
    s = native().J2CSink(2, 1 << 16)
    body = _tera(300)[:-2]
    cut = (len(body) // 104 // 2) * 104
    assert s.consume(0, body[:cut]) == 0
    assert s.consume(0, body[cut:] + EOF_MARK) == 0
    assert s.records(0) == 300 and s.eof(0) and not s.eof(1)
    assert s.bytes(0) == len(body) + 2 and s.buffers(0) == 2


def test_framing_errors_and_data_after_eof():
    n = native()
    s = n.J2CSink(1, 1 << 16)
    body = _tera(10)[:-2]
    assert s.consume(0, body[:-5]) != 0  # a record cut in the middle
    s2 = n.J2CSink(1, 1 << 16)
    assert s2.consume(0, EOF_MARK) == 0
    assert s2.consume(0, body) != 0      # data after the EOF marker
    s3 = n.J2CSink(1, 64)
    assert s3.consume(0, body) != 0      # longer than kv_buf


def test_multibyte_vint_lengths():
    recs = [(text(b"k%04d" % i), os.urandom(300 + i)) for i in range(20)]  # values >= 128 bytes
    body = encode_stream(recs)
    s = native().J2CSink(1, 1 << 16)
    assert s.consume(0, body) == 0
    assert s.records(0) == 20 and s.eof(0)


def test_key_order_check():
    n = native()
    good = _tera(200)[:-2]
    s = n.J2CSink(1, 1 << 16)
    s.set_check_order(True)
    assert s.consume(0, good + EOF_MARK) == 0
    assert s.order_errors(0) == 0
    recs = [(text(b"b"), b"1"), (text(b"a"), b"2")]
    s2 = n.J2CSink(1, 1 << 16)
    s2.set_check_order(True)
    assert s2.consume(0, encode_stream(recs)) == 0
    assert s2.order_errors(0) == 1


@pytest.mark.parametrize("reps", [1, 50])
def test_repeat_consume_is_additive(reps):
    s = native().J2CSink(1, 1 << 20)
    body = _tera(1000)[:-2]
    assert s.consume(0, body, reps) == 0
    assert s.records(0) == 1000 * reps
