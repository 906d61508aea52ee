"""Python views of the native data-path operations.

merge_runs(runs, key_class, device="gpu"|"cpu") merges sorted IFile runs (byte strings, each the
raw partition stream of one map output) and returns (merged record bytes, buffer cut offsets).
The GPU path runs the HIP kernels F1 (record index), F2 (key normalize), F3 (merge-path merge
tree) and F4 (scan + gather) of csrc/gpu; the CPU path is the reference heap merge. There is no
silent fallback: device="gpu" raises when no HIP device or extension is available.
"""
from __future__ import annotations

from .._native import native

EOF_MARKER = b"\xff\xff"
last_stats: dict = {}  # timing of the most recent merge_runs call (device merge excludes H2D/D2H)


def merge_runs(runs: list[bytes], key_class: str, device: str = "gpu", kv_buf: int = 1 << 20,
               gpu_index: int = 0):
    n = native()
    if device == "gpu":
        if n.device_count() <= 0:
            raise RuntimeError("merge_runs(device='gpu'): no HIP device visible")
        merged, cuts, _records, _passes, merge_ms, serial = n.gpu_merge_runs(list(runs), key_class, kv_buf - 2,
                                                                             gpu_index)
        last_stats.update(device="gpu", records=_records, passes=_passes, merge_ms=merge_ms, f1_serial_runs=serial)
        return merged, cuts
    if device == "cpu":
        out, lens = n.cpu_merge(list(runs), key_class, kv_buf)
        # cpu_merge already appended the EOF marker and packed greedily
        body = out[:-2]
        cuts, pos = [0], 0
        for ln in lens:
            pos = min(pos + ln, len(body))
            if pos != cuts[-1]:
                cuts.append(pos)
        return body, cuts
    raise ValueError(f"unknown device {device!r}")


def buffers(merged: bytes, cuts: list[int]) -> list[bytes]:
    """Split a merged stream at the cut offsets into delivery buffers, EOF in the last one."""
    out = [merged[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    if out:
        out[-1] += EOF_MARKER
    else:
        out = [EOF_MARKER]
    return out
