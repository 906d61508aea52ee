"""Native J2C consumer (the stand-in for the Java reducer's J2CQueue): every buffer is copied into a
KVBuf and walked by its VInt lengths; framing errors, data after EOF and key order are detected.
Both threading models: the plugin's (dataFromUda copies on the delivering thread, the reduce task's
own thread walks the two KVBufs in turn) and inline (one thread copies and walks)."""
import os
import threading

import pytest

from uda_amd import native
from uda_amd.utils.ifile import encode_stream, text

EOF_MARK = b"\xff\xff"
MODES = [True, False]


def _tera(n, seed=1):
    rnd = __import__("random").Random(seed)
    keys = sorted(bytes(rnd.getrandbits(8) for _ in range(10)) for _ in range(n))
    return encode_stream([(text(k), text(b"V" * 90)) for k in keys])


def _feed(s, r, *bufs):
    """dataFromUda for every buffer, then wait for the walks; the first error code seen."""
    rc = 0
    for b in bufs:
        rc = rc or s.consume(r, b)
    s.flush()
    return rc or s.error(r)


@pytest.mark.parametrize("threaded", MODES)
def test_counts_records_and_eof(threaded):
    s = native().J2CSink(2, 1 << 16, threaded)
    assert s.threaded == threaded
    body = _tera(300)[:-2]
    cut = (len(body) // 104 // 2) * 104
    assert _feed(s, 0, body[:cut], body[cut:] + EOF_MARK) == 0
    assert s.records(0) == 300 and s.eof(0) and not s.eof(1)
    assert s.bytes(0) == len(body) + 2 and s.buffers(0) == 2


@pytest.mark.parametrize("threaded", MODES)
def test_framing_errors_and_data_after_eof(threaded):
    n = native()
    s = n.J2CSink(1, 1 << 16, threaded)
    body = _tera(10)[:-2]
    assert _feed(s, 0, body[:-5]) != 0  # a record cut in the middle
    s2 = n.J2CSink(1, 1 << 16, threaded)
    assert _feed(s2, 0, EOF_MARK) == 0
    assert _feed(s2, 0, body) != 0      # data after the EOF marker
    s3 = n.J2CSink(1, 64, threaded)
    assert s3.consume(0, body) != 0     # longer than kv_buf: refused by dataFromUda itself


@pytest.mark.parametrize("threaded", MODES)
def test_multibyte_vint_lengths(threaded):
    recs = [(text(b"k%04d" % i), os.urandom(300 + i)) for i in range(20)]  # values >= 128 bytes
    body = encode_stream(recs)
    s = native().J2CSink(1, 1 << 16, threaded)
    assert _feed(s, 0, body) == 0
    assert s.records(0) == 20 and s.eof(0)


@pytest.mark.parametrize("threaded", MODES)
def test_key_order_check(threaded):
    n = native()
    good = _tera(200)[:-2]
    s = n.J2CSink(1, 1 << 16, threaded)
    s.set_check_order(True)
    assert _feed(s, 0, good + EOF_MARK) == 0
    assert s.order_errors(0) == 0
    recs = [(text(b"b"), b"1"), (text(b"a"), b"2")]
    s2 = n.J2CSink(1, 1 << 16, threaded)
    s2.set_check_order(True)
    assert _feed(s2, 0, encode_stream(recs)) == 0
    assert s2.order_errors(0) == 1


@pytest.mark.parametrize("threaded", MODES)
@pytest.mark.parametrize("reps", [1, 50])
def test_repeat_consume_is_additive(reps, threaded):
    s = native().J2CSink(1, 1 << 20, threaded)
    body = _tera(1000)[:-2]
    assert s.consume(0, body, reps) == 0
    s.flush()
    assert s.records(0) == 1000 * reps and s.buffers(0) == reps


def test_threaded_handoff_many_buffers_many_reducers():
    """Several delivering threads (one per reducer), hundreds of buffers each through the two-KVBuf
    handshake: every record walked once, in order, EOF last; reset() between passes."""
    n = native()
    R = 4
    s = n.J2CSink(R, 1 << 16, True)
    s.set_check_order(True)
    body = _tera(2000, seed=3)[:-2]
    pieces = [body[i:i + 104 * 37] for i in range(0, len(body), 104 * 37)]
    for _ in range(2):
        s.reset()
        errs = []

        def deliver(r):
            rc = 0
            for p in pieces:
                rc = rc or s.consume(r, p)
            rc = rc or s.consume(r, EOF_MARK)
            errs.append(rc)

        ts = [threading.Thread(target=deliver, args=(r,)) for r in range(R)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        s.flush()
        assert errs == [0] * R
        for r in range(R):
            assert s.records(r) == 2000 and s.eof(r) and s.error(r) == 0 and s.order_errors(r) == 0
            assert s.buffers(r) == len(pieces) + 1
