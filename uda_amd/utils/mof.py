"""Map-output files (MOFs) in Hadoop's on-disk layout, for tests, tools and the loopback configs.

file.out holds one IFile partition per reducer back to back (optionally block-compressed);
file.out.index holds, per partition, three big-endian longs {startOffset, rawLength, partLength}
followed by a CRC32 of those bytes as a big-endian long (Hadoop SpillRecord). The index record is
the tuple the provider's getPathUda callback returns (IndexRecordBridge.java:26-34).
"""
from __future__ import annotations

import os
import struct
import zlib

from .._native import native

CODECS = {None: 0, "snappy": 1, "lzo": 2}
CODEC_CLASSES = {
    None: None,
    "snappy": "org.apache.hadoop.io.compress.SnappyCodec",
    "lzo": "com.hadoop.compression.lzo.LzoCodec",
}


def encode_partitions(partitions: list[bytes], codec: str | None = None, block_size: int = 256 * 1024):
    """Returns (file_bytes, index) with index = [(start, raw_len, part_len)]."""
    data = bytearray()
    index = []
    for p in partitions:
        raw = len(p)
        body = native().block_compress(CODECS[codec], p, block_size) if codec else p
        index.append((len(data), raw, len(body)))
        data += body
    return bytes(data), index


def write_index(path: str, index) -> None:
    body = b"".join(struct.pack(">qqq", *rec) for rec in index)
    with open(path, "wb") as f:
        f.write(body)
        f.write(struct.pack(">q", zlib.crc32(body) & 0xFFFFFFFF))


def read_index(path: str):
    with open(path, "rb") as f:
        blob = f.read()
    body, crc = blob[:-8], struct.unpack(">q", blob[-8:])[0]
    if zlib.crc32(body) & 0xFFFFFFFF != crc:
        raise ValueError(f"index checksum mismatch in {path}")
    return [struct.unpack(">qqq", body[i:i + 24]) for i in range(0, len(body), 24)]


def write_mof(directory: str, map_id: str, partitions: list[bytes], codec: str | None = None,
              block_size: int = 256 * 1024) -> tuple[str, list]:
    """Write <directory>/<map_id>/file.out(+.index). Returns (file.out path, index)."""
    d = os.path.join(directory, map_id)
    os.makedirs(d, exist_ok=True)
    data, index = encode_partitions(partitions, codec, block_size)
    out = os.path.join(d, "file.out")
    with open(out, "wb") as f:
        f.write(data)
    write_index(out + ".index", index)
    return out, index
