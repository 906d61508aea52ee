"""F6 device block decode (Snappy / LZO1X) against the original bytes and the host decoders.

Inputs cover incompressible data (long literals), short-period repeats (overlapping copies with
offset < length), long non-overlapping back-references at odd alignments (the 16-byte vector
copies), IFile streams, empty blocks and streams, multi-chunk Snappy blocks, and Snappy
streams from an independent encoder (pyarrow's libsnappy) when available.
"""
import os
import random
import struct

import pytest

from uda_amd.utils import datagen

pytestmark = pytest.mark.gpu

SNAPPY, LZO = 1, 2


def _payloads():
    rng = random.Random(11)
    yield "random", os.urandom(300_000)
    yield "period1", b"\x00" * 100_000
    yield "period3", b"abc" * 50_000 + b"x"
    yield "mixed", b"".join(
        (os.urandom(rng.randint(1, 300)) if rng.random() < 0.5 else bytes([rng.randrange(256)]) * rng.randint(1, 900))
        for _ in range(600))
    base = os.urandom(5000)  # slices of one text: long non-overlapping back-references at odd alignments
    yield "slices", b"".join(base[o:o + n] for o, n in ((rng.randrange(4700), rng.randint(4, 300)) for _ in range(2000)))
    yield "ifile", datagen.streams(datagen.secondary_sort(3, 1, 3000, seed=2))[0][0]
    yield "tiny", b"q"
    yield "empty", b""


@pytest.mark.parametrize("codec", [SNAPPY, LZO], ids=["snappy", "lzo"])
@pytest.mark.parametrize("block", [4096, 65536, 262144])
def test_device_decode_roundtrip(require_gpu, native, codec, block):
    names, raws, streams = [], [], []
    for name, raw in _payloads():
        names.append(name)
        raws.append(raw)
        streams.append(native.block_compress(codec, raw, block))
    outs, blocks, _ms = native.gpu_block_decode("snappy" if codec == SNAPPY else "lzo", streams)
    assert blocks == sum((len(r) + block - 1) // block for r in raws)
    for name, raw, out, st in zip(names, raws, outs, streams):
        assert out == raw, name
        assert out == native.block_decompress(codec, st, 1 << 20), name


def test_snappy_multichunk_blocks_and_empty_blocks(require_gpu, native):
    parts = [os.urandom(5000), b"z" * 7000, b"hello world " * 300]
    chunks = [native.snappy_compress(p) for p in parts]
    raw = b"".join(parts)
    block = struct.pack(">I", len(raw)) + b"".join(struct.pack(">I", len(c)) + c for c in chunks)
    stream = struct.pack(">I", 0) + block + struct.pack(">I", 0) + block
    outs, blocks, _ = native.gpu_block_decode("snappy", [stream, b""])
    assert outs[0] == raw + raw and outs[1] == b""
    assert blocks == 2


def test_snappy_from_independent_encoder(require_gpu, native):
    pa = pytest.importorskip("pyarrow")
    raws = [datagen.streams(datagen.wordcount(2, 1, 20000, seed=3))[0][0], os.urandom(70000), b"ab" * 90000]
    streams = []
    for raw in raws:
        s = b""
        for off in range(0, len(raw), 131072):
            piece = raw[off:off + 131072]
            c = pa.compress(piece, codec="snappy", asbytes=True)
            s += struct.pack(">II", len(piece), len(c)) + c
        streams.append(s)
    outs, _, _ = native.gpu_block_decode("snappy", streams)
    assert outs == raws


@pytest.mark.parametrize("codec", ["snappy", "lzo"])
def test_corrupt_block_raises(require_gpu, native, codec):
    raw = b"abcdefgh" * 4000 + os.urandom(1000)
    st = bytearray(native.block_compress(SNAPPY if codec == "snappy" else LZO, raw, 65536))
    # break a back-reference: overwrite the body of the first block with 0xFF bytes
    for i in range(12, min(len(st), 60)):
        st[i] = 0xFF
    with pytest.raises(Exception, match="corrupt|framing"):
        native.gpu_block_decode(codec, [bytes(st)])


@pytest.mark.parametrize("codec", ["snappy", "lzo"])
def test_consumer_gpu_backend_decodes_on_device(require_gpu, tmp_path, codec):
    from uda_amd.bridge import UdaProvider, run_reduce
    from uda_amd.utils.mof import write_mof
    p = UdaProvider()
    try:
        maps = datagen.wordcount(num_maps=6, reducers=2, words_per_map=5000, seed=13)
        ids = []
        for i, parts in enumerate(datagen.streams(maps)):
            mid = f"attempt_d{codec}_m_{i:06d}_0"
            path, _ = write_mof(str(tmp_path), mid, parts, codec=codec)
            p.add_mof_file(f"job_d{codec}", mid, path)
            ids.append(mid)
        recs, st, _ = run_reduce("h", f"job_d{codec}", ids, 0, datagen.TEXT, codec=codec,
                                 conf={"mapred.uda.merge.backend": "gpu"}, kv_buf_size=8192)
        assert st["device_decoded_blocks"] > 0
        want = sorted((kv for m in maps for kv in m[0]), key=datagen.sort_key(datagen.TEXT))
        kf = datagen.sort_key(datagen.TEXT)
        assert [kf(kv) for kv in recs] == [kf(kv) for kv in want]
        assert sorted(recs) == sorted(want)
    finally:
        p.close()


def test_lzo1x_spec_vectors_on_device(require_gpu, native):
    """The device LZO1X decoder on hand-assembled streams (not produced by our encoder)."""
    from tests.lzo_vectors import VECTORS, hadoop_block
    streams = [hadoop_block(want, st) for _, st, want in VECTORS]
    outs, blocks, _ = native.gpu_block_decode("lzo", streams)
    assert blocks == len(VECTORS)
    assert outs == [want for _, _, want in VECTORS]


@pytest.mark.parametrize("env", [{}, {"UDA_DECODE_WINDOW": "reg"}, {"UDA_DECODE_WINDOW": "lds"}, {"UDA_LZO_LANE": "1"}],
                         ids=["wave-lean", "wave-register-window", "wave-lds-window", "lane-per-block"])
@pytest.mark.parametrize("codec", ["lzo", "snappy"])
def test_decode_kernels_agree_on_terasort_records(require_gpu, native, monkeypatch, env, codec):
    """Every device decode kernel -- one wave per block parsing from a register window (LZO: the lean
    parse by default, the per-byte parse with "reg"; Snappy: the register window for both) or from the LDS
    window of round 5, and for LZO one lane per block -- decodes TeraSort-shaped IFile records
    (random keys, 26-letter values: streams of many 3-4 byte tokens) and every other payload to the
    original bytes, and reports a corrupt block."""
    if codec == "snappy" and "UDA_LZO_LANE" in env:
        pytest.skip("LZO only")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cid = LZO if codec == "lzo" else SNAPPY
    tera = datagen.streams(datagen.terasort(2, 1, 6000, seed=5))[0][0]
    raws = [tera] + [raw for _, raw in _payloads()]
    for block in (4096, 262144):
        streams = [native.block_compress(cid, raw, block) for raw in raws]
        outs, blocks, _ms = native.gpu_block_decode(codec, streams)
        assert blocks == sum((len(r) + block - 1) // block for r in raws)
        assert all(o == r for o, r in zip(outs, raws))
    raw = b"abcdefgh" * 4000 + os.urandom(1000)
    st = bytearray(native.block_compress(cid, raw, 65536))
    for i in range(12, min(len(st), 60)):  # a broken back-reference, as test_corrupt_block_raises
        st[i] = 0xFF
    with pytest.raises(Exception, match="corrupt|framing"):
        native.gpu_block_decode(codec, [bytes(st)])
