"""In-tree Snappy / LZO1X codecs and Hadoop block framing.

Snappy parity is pinned against pyarrow's Snappy (an independent implementation) in both
directions. LZO1X: no independent LZO implementation is importable here (liblzo2 is absent), so its
parity with liblzo2 is unpinned; it is checked by round trips through our encoder (which emits
literal runs, M2/M3/M4 matches, long-length extensions and trailing-literal states) and by
rejecting corrupted streams.
"""
import os
import random

import pytest


def samples():
    rng = random.Random(11)
    yield b""
    yield b"a"
    yield b"abcd" * 1000
    yield os.urandom(5000)
    yield bytes(rng.choice(b"ACGT") for _ in range(100000))
    yield b"".join(b"key%08d\tvalue%d\n" % (i, i % 97) for i in range(5000))
    yield b"\x00" * 70000 + b"x" + b"\x00" * 300   # long matches -> length extensions


@pytest.mark.parametrize("idx", range(7))
def test_snappy_vs_pyarrow(native, idx):
    pa = pytest.importorskip("pyarrow")
    d = list(samples())[idx]
    ours = native.snappy_compress(d)
    assert pa.decompress(ours, decompressed_size=len(d), codec="snappy", asbytes=True) == d
    theirs = pa.compress(d, codec="snappy", asbytes=True)
    assert native.snappy_decompress(theirs, len(d)) == d


@pytest.mark.parametrize("idx", range(7))
def test_lzo_roundtrip(native, idx):
    d = list(samples())[idx]
    c = native.lzo1x_compress(d)
    assert native.lzo1x_decompress(c, len(d)) == d


def test_lzo_far_offsets(native):
    # repeats at distances > 16 KiB exercise the M4 (offset 0x4000..0xbfff) encoding
    rng = random.Random(5)
    block = bytes(rng.getrandbits(8) for _ in range(20000))
    d = block + os.urandom(100) + block[:5000] + os.urandom(30000) + block[1000:9000]
    assert native.lzo1x_decompress(native.lzo1x_compress(d), len(d)) == d


@pytest.mark.parametrize("codec", ["snappy", "lzo"])
def test_corrupt_streams_rejected(native, codec):
    d = b"hello world, hello world, hello hello hello" * 50
    comp = getattr(native, f"{'snappy' if codec == 'snappy' else 'lzo1x'}_compress")(d)
    dec = getattr(native, f"{'snappy' if codec == 'snappy' else 'lzo1x'}_decompress")
    with pytest.raises(ValueError):
        dec(comp[: len(comp) // 2], len(d))
    with pytest.raises(ValueError):
        dec(comp, len(d) // 2)  # output too small


@pytest.mark.parametrize("codec,feed", [(1, 1), (1, 7), (1, 100000), (2, 3), (2, 65536)])
def test_block_framing_incremental(native, codec, feed):
    d = b"".join(os.urandom(10) + b"common-suffix-%d" % (i % 13) for i in range(20000))
    framed = native.block_compress(codec, d, 4096 + 17)
    assert native.block_decompress(codec, framed, feed) == d


def test_block_truncated(native):
    framed = native.block_compress(1, b"x" * 100000, 8192)
    with pytest.raises(ValueError):
        native.block_decompress(1, framed[:-3], 1000)


def test_codec_classes(native):
    assert native.codec_from_class("org.apache.hadoop.io.compress.SnappyCodec") == 1
    assert native.codec_from_class("com.hadoop.compression.lzo.LzoCodec") == 2
    assert native.codec_from_class("null") == 0
    assert native.codec_from_class("org.apache.hadoop.io.compress.GzipCodec") == -1


@pytest.mark.parametrize("backend", ["", "threadpool"])
def test_async_io_backends(native, tmp_path, backend):
    name, ok = native.aio_selftest(str(tmp_path / "aio.bin"), (5 << 20) + 123, backend)
    assert ok
    if backend == "threadpool":
        assert name == "threadpool"


@pytest.mark.parametrize("name", [v[0] for v in __import__("tests.lzo_vectors", fromlist=["VECTORS"]).VECTORS])
def test_lzo1x_spec_vectors(native, name):
    """Hand-assembled LZO1X streams (independent of the in-tree encoder) decode to the output the
    format defines, through the raw decoder and the Hadoop block framing."""
    from tests.lzo_vectors import VECTORS, hadoop_block
    stream, want = {v[0]: (v[1], v[2]) for v in VECTORS}[name]
    assert native.lzo1x_decompress(stream, len(want)) == want
    assert native.block_decompress(2, hadoop_block(want, stream), 7) == want


def test_lzo_lane_decoder_on_the_host(native):
    """The LZO1X per-lane decode of the device lane kernel (one lane per block), run on the host: every
    payload shape (TeraSort records, incompressible, period-1/3 repeats, odd-alignment back-references,
    IFile streams) at every block size decodes to the original; a broken back-reference is refused."""
    import os
    import random

    from uda_amd.utils import datagen
    rng = random.Random(11)
    base = os.urandom(5000)
    pays = [datagen.streams(datagen.terasort(2, 1, 6000, seed=5))[0][0], os.urandom(300_000), b"\x00" * 100_000,
            b"abc" * 50_000 + b"x", b"q", b"",
            b"".join((os.urandom(rng.randint(1, 300)) if rng.random() < 0.5 else bytes([rng.randrange(256)]) *
                      rng.randint(1, 900)) for _ in range(600)),
            b"".join(base[o:o + k] for o, k in ((rng.randrange(4700), rng.randint(4, 300)) for _ in range(2000))),
            datagen.streams(datagen.secondary_sort(3, 1, 3000, seed=2))[0][0]]
    for block in (4096, 65536, 262144):
        for p in pays:
            assert native.lzo_lane_decode_host(native.block_compress(2, p, block), len(p)) == p
    st = bytearray(native.block_compress(2, b"abcdefgh" * 4000 + os.urandom(1000), 65536))
    for i in range(12, 60):
        st[i] = 0xFF
    with pytest.raises(RuntimeError, match="corrupt"):
        native.lzo_lane_decode_host(bytes(st), 40_000)
