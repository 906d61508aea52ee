"""Hadoop IFile record codec and a J2CQueue-equivalent buffer reader (pure Python, for tests and
small tools; the hot paths are native).

Formats: a record is VInt keyLen, VInt valLen, key bytes, value bytes; a stream
ends with VInt(-1) VInt(-1). VInt is Hadoop's zero-compressed encoding
(src/CommUtils/IOUtility.cc:167-196). The merged output reaches the reducer as buffers of whole
records; J2CQueue (plugins/shared/com/mellanox/hadoop/mapred/UdaPlugin.java:435-538) moves to the
next buffer when its position reaches len-1 and stops at a negative length.
"""
from __future__ import annotations

EOF_MARKER = b"\xff\xff"


def vint_encode(v: int) -> bytes:
    if -112 <= v <= 127:
        return bytes([v & 0xFF])
    length = -112
    if v < 0:
        v ^= -1
        length = -120
    t = v
    while t != 0:
        t >>= 8
        length -= 1
    n = -(length + 120) if length < -120 else -(length + 112)
    return bytes([length & 0xFF]) + v.to_bytes(n, "big")


def vint_decode(buf: bytes | memoryview, pos: int = 0) -> tuple[int, int]:
    """Returns (value, bytes consumed). Raises EOFError on truncation."""
    if pos >= len(buf):
        raise EOFError
    b = buf[pos]
    b = b - 256 if b > 127 else b
    if b >= -112:
        return b, 1
    neg = b < -120
    n = (-120 - b) if neg else (-112 - b)
    if pos + 1 + n > len(buf):
        raise EOFError
    v = int.from_bytes(bytes(buf[pos + 1:pos + 1 + n]), "big")
    if neg:
        v ^= -1
    return v, n + 1


def encode_record(key: bytes, val: bytes) -> bytes:
    return vint_encode(len(key)) + vint_encode(len(val)) + key + val


def text(s: bytes) -> bytes:
    """Serialize bytes as a Hadoop Text writable (VInt length + bytes)."""
    return vint_encode(len(s)) + s


def encode_stream(records, eof: bool = True) -> bytes:
    out = bytearray()
    for k, v in records:
        out += encode_record(k, v)
    if eof:
        out += EOF_MARKER
    return bytes(out)


def decode_stream(buf: bytes, require_eof: bool = True):
    """Decode a full IFile stream into [(key, value)]."""
    out = []
    pos = 0
    while True:
        if pos >= len(buf):
            if require_eof:
                raise ValueError("stream ended without EOF marker")
            return out
        kl, a = vint_decode(buf, pos)
        vl, b = vint_decode(buf, pos + a)
        pos += a + b
        if kl < 0 or vl < 0:
            return out
        out.append((bytes(buf[pos:pos + kl]), bytes(buf[pos + kl:pos + kl + vl])))
        pos += kl + vl


class J2CQueueReader:
    """Consumes delivered buffers the way J2CQueue does and checks the framing contract:
    every buffer holds whole records, is at most `max_len` bytes, and the stream ends with EOF."""

    def __init__(self, max_len: int = 1 << 20):
        self.max_len = max_len
        self.records: list[tuple[bytes, bytes]] = []
        self.buffers = 0
        self.eof = False

    def feed(self, buf: bytes) -> None:
        if self.eof:
            raise AssertionError("buffer delivered after EOF")
        if len(buf) > self.max_len:
            raise AssertionError(f"buffer of {len(buf)} bytes exceeds {self.max_len}")
        self.buffers += 1
        pos = 0
        while pos < len(buf) - 1:
            kl, a = vint_decode(buf, pos)
            vl, b = vint_decode(buf, pos + a)
            pos += a + b
            if kl < 0 or vl < 0:
                self.eof = True
                if pos != len(buf):
                    raise AssertionError("bytes after EOF marker")
                return
            if pos + kl + vl > len(buf):
                raise AssertionError("record split across buffers")
            self.records.append((bytes(buf[pos:pos + kl]), bytes(buf[pos + kl:pos + kl + vl])))
            pos += kl + vl
        if pos != len(buf):
            raise AssertionError("trailing partial record in buffer")
