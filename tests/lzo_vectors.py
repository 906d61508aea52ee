"""LZO1X streams built by hand from the format (not by our encoder): the decoders are checked
against the LZO1X instruction semantics (lzo1x_d.ch behaviour, as documented in the LZO source):

  first byte > 17        : literal run of (b - 17) bytes
  0..15 (literal state)  : literal run of t + 3 (t == 0: 15 + extension bytes, 255 per zero byte)
  16..31  M4             : distance 16384 + ..., or the end marker 0x11 0x00 0x00
  32..63  M3             : length (t & 31) + 2, distance 1 + (b0 >> 2) + (b1 << 6)
  64..255 M2             : length (t >> 5) + 1, distance 1 + ((t >> 2) & 7) + (b << 3)
  low 2 bits of the last distance byte: 0..3 literals that follow the match
"""
EOF_MARKER = bytes([0x11, 0x00, 0x00])
LIT20 = bytes(range(65, 85))

VECTORS = [
    # (name, stream, expected output)
    ("literals_only", bytes([17 + 3]) + b"abc" + EOF_MARKER, b"abc"),
    ("m3_overlapping_copy", bytes([17 + 3]) + b"abc" + bytes([0x20 | 7, 2 << 2, 0x00]) + EOF_MARKER,
     b"abc" + b"abcabcabc"),
    ("m2_match", bytes([17 + 4]) + b"abcd" + bytes([(3 << 5) | (3 << 2), 0x00]) + EOF_MARKER, b"abcdabcd"),
    ("m2_trailing_literals", bytes([17 + 4]) + b"abcd" + bytes([(3 << 5) | (3 << 2) | 2, 0x00]) + b"XY" + EOF_MARKER,
     b"abcdabcdXY"),
    ("long_literal_run_extension", bytes([17 + 3]) + b"abc" + bytes([0x20 | 7, 2 << 2, 0x00]) + bytes([0x00, 0x02])
     + LIT20 + EOF_MARKER, b"abc" + b"abcabcabc" + LIT20),
    ("first_run_238_literals", bytes([17 + 238]) + bytes(range(238)) + EOF_MARKER, bytes(range(238))),
]


def hadoop_block(raw: bytes, payload: bytes) -> bytes:
    """Hadoop BlockCompressorStream framing: [u32 BE raw][u32 BE compressed][payload]."""
    return len(raw).to_bytes(4, "big") + len(payload).to_bytes(4, "big") + payload
