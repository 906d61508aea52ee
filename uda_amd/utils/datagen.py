"""Synthetic map outputs for the BASELINE configs (host-side, for tests and CPU configs).

* TeraSort: 10-byte random keys, 90-byte values, Text/Text (104-byte IFile records).
* WordCount: Text word -> IntWritable count, Zipf-skewed vocabulary (uda_standalone wordcount).
* Secondary sort: variable-length Text keys sharing long common prefixes (defeats fixed-width key
  prefixes, forcing full comparisons) with skewed partition sizes.
Each generator returns per-map lists of per-reducer sorted record lists [(key, value)], so the
merge inputs are sorted runs exactly like a map task's spill.
"""
from __future__ import annotations

import random

from .._native import native
from .ifile import encode_stream, text

TEXT = "org.apache.hadoop.io.Text"
INT = "org.apache.hadoop.io.IntWritable"
BYTES = "org.apache.hadoop.io.BytesWritable"
LONG = "org.apache.hadoop.io.LongWritable"


def sort_key(key_class: str):
    """Python key function matching the native comparator for a key class."""
    if key_class == TEXT:
        def f(kv):
            k = kv[0]
            n = native().vint_decode_size(k[0] - 256 if k[0] > 127 else k[0]) if k else 0
            return k[n:]
        return f
    if key_class in (BYTES, "org.apache.hadoop.hbase.io.ImmutableBytesWritable"):
        return lambda kv: kv[0][4:]
    return lambda kv: kv[0]


def partition_of(key: bytes, reducers: int) -> int:
    h = 0
    for b in key:
        h = (h * 31 + b) & 0x7FFFFFFF
    return h % reducers


def _finish(maps: list[list[list]], key_class: str):
    kf = sort_key(key_class)
    return [[sorted(part, key=kf) for part in m] for m in maps]


def terasort(num_maps: int, reducers: int, rows_per_map: int, seed: int = 1):
    rng = random.Random(seed)
    maps = []
    for _ in range(num_maps):
        parts = [[] for _ in range(reducers)]
        for _ in range(rows_per_map):
            k = bytes(rng.getrandbits(8) for _ in range(10))
            v = bytes(rng.choice(b"ABCDEFGHIJKLMNOPQRSTUVWXYZ") for _ in range(90))
            parts[k[0] * reducers // 256].append((text(k), text(v)))
        maps.append(parts)
    return _finish(maps, TEXT)


def wordcount(num_maps: int, reducers: int, words_per_map: int, vocab: int = 5000, seed: int = 2):
    rng = random.Random(seed)
    words = [("w%06d" % i).encode() for i in range(vocab)]
    weights = [1.0 / (i + 1) for i in range(vocab)]  # Zipf-like skew
    maps = []
    for _ in range(num_maps):
        counts: dict[bytes, int] = {}
        for w in rng.choices(words, weights, k=words_per_map):
            counts[w] = counts.get(w, 0) + 1  # map-side combiner
        parts = [[] for _ in range(reducers)]
        for w, c in counts.items():
            parts[partition_of(w, reducers)].append((text(w), c.to_bytes(4, "big")))
        maps.append(parts)
    return _finish(maps, TEXT)


def secondary_sort(num_maps: int, reducers: int, rows_per_map: int, seed: int = 3, skew: float = 0.6):
    rng = random.Random(seed)
    prefixes = [b"user/%04d/session/" % i + b"x" * rng.randint(0, 40) for i in range(64)]
    maps = []
    for _ in range(num_maps):
        parts = [[] for _ in range(reducers)]
        for _ in range(rows_per_map):
            p = prefixes[min(int(rng.paretovariate(1.2)) - 1, 63)]
            k = p + b"%08d" % rng.randint(0, 10 ** 6)
            v = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 120)))
            r = 0 if rng.random() < skew else partition_of(k, reducers)
            parts[r].append((text(k), text(v)))
        maps.append(parts)
    return _finish(maps, TEXT)


def bytes_writable(num_maps: int, reducers: int, rows_per_map: int, seed: int = 4):
    """BytesWritable keys (4-byte big-endian length + raw bytes, any byte values, shared prefixes)."""
    rng = random.Random(seed)
    maps = []
    for _ in range(num_maps):
        parts = [[] for _ in range(reducers)]
        for _ in range(rows_per_map):
            body = bytes([rng.choice((0, 1, 255))]) * rng.randint(0, 12) + bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 20)))
            k = len(body).to_bytes(4, "big") + body
            parts[partition_of(k, reducers)].append((k, bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 40)))))
        maps.append(parts)
    return _finish(maps, BYTES)


def streams(maps) -> list[list[bytes]]:
    """Encode per-map per-reducer record lists into IFile partition streams (with EOF)."""
    return [[encode_stream(part) for part in m] for m in maps]
