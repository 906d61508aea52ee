"""GPU: F8 map-side sort (`csrc/gpu/radix.hip`, LSD radix sort on the 10-byte TeraSort key + gather).

Numerics oracle: Python's stable `sorted` of the same records by their key bytes. Equal keys carry
different values, so the comparison also checks that the sort is stable (LSD needs every pass stable).
"""
import numpy as np
import pytest

from uda_amd.parallel.dist import DistContext

pytestmark = pytest.mark.gpu

REC = 104


def _records(n, seed, key_values=None):
    """n TeraSort IFile records: VInt(11) VInt(91) VInt(10) key[10] VInt(90) value[90]."""
    rng = np.random.default_rng(seed)
    r = np.zeros((n, REC), dtype=np.uint8)
    r[:, 0], r[:, 1], r[:, 2], r[:, 13] = 0x0B, 0x5B, 0x0A, 0x5A
    if key_values is None:
        r[:, 3:13] = rng.integers(0, 256, size=(n, 10), dtype=np.uint8)
    else:  # few distinct keys: long runs of equal keys (stability)
        keys = rng.integers(0, 256, size=(key_values, 10), dtype=np.uint8)
        r[:, 3:13] = keys[rng.integers(0, key_values, size=n)]
    r[:, 14:] = rng.integers(ord("A"), ord("Z") + 1, size=(n, 90), dtype=np.uint8)
    return r


def _oracle(r):
    order = sorted(range(len(r)), key=lambda i: bytes(r[i, 3:13]))
    return r[order].tobytes()


@pytest.mark.parametrize("staged", [False, True])
@pytest.mark.parametrize("n,distinct", [(1, None), (2, None), (255, None), (4096, None), (4097, None),
                                        (100_003, None), (50_000, 3), (70_000, 1)])
def test_sort_fixed_matches_stable_python_sort(require_gpu, native, n, distinct, staged):
    """staged=False: records sorted where they are; staged=True: the engine's map-sort layout (unsorted
    records in the sort workspace, gathered sorted into the store)."""
    r = _records(n, seed=n, key_values=distinct)
    out, ms = native.gpu_sort_fixed(r.tobytes(), staged=staged)
    assert out == _oracle(r)
    assert ms >= 0


def test_sort_fixed_adversarial_key_bytes(require_gpu, native):
    # keys that differ only in the last byte, only in the first byte, and 0x00/0xFF extremes
    n = 3 * 4096 + 17
    r = _records(n, seed=7)
    r[: n // 3, 3:12] = 0x00
    r[n // 3: 2 * n // 3, 4:13] = 0xFF
    r[2 * n // 3:, 3:13] = np.where(np.arange(10) % 2 == 0, 0x00, 0xFF).astype(np.uint8)
    out, _ = native.gpu_sort_fixed(r.tobytes())
    assert out == _oracle(r)


@pytest.mark.parametrize("store", ["hbm", "host"])
def test_terasort_with_map_side_sort(require_gpu, store):
    """Unsorted map input, sorted per partition on the device at setup; the shuffle's validated step
    checks key order per reducer and the record checksum against the generated records."""
    from uda_amd.models.terasort import TeraSortConfig, TeraSortShuffle
    cfg = TeraSortConfig(rows_per_gpu=300_000, maps_per_rank=6, rounds=3, reducers=2, validate=True,
                         sample_every=64, map_sort=True, store=store,
                         kv_buf_bytes=64 << 10, d2h_piece_bytes=256 << 10)
    j = TeraSortShuffle(DistContext(), cfg, device=0)
    j.setup()
    assert j.job.map_sort_ms > 0
    st = j.step()
    j.check(st)
    assert st["order_errors"] == 0
    assert st["checksum"] == j.expected_checksum
    assert st["records"] == 300_000
