"""Key-range round planning (the TeraSort range-partition sampler's role).

GPU d owns a key range, cut into C = reducers x rounds cells: cell c holds the keys in
[bound(d, c-1), bound(d, c)); reducer i owns cells [i*rounds, (i+1)*rounds) and round q ships cell
i*rounds + q of every reducer. Bounds are quantiles of a key sample gathered from every rank, so
cells carry near-equal volume even under key skew. Ties go to the upper cell (lower_bound).
"""
from __future__ import annotations

import numpy as np


def quantile_bounds(samples: np.ndarray, rounds: int) -> np.ndarray:
    """samples: (n, 2) uint64 (hi, lo). Returns (rounds-1, 2) uint64 ascending bounds."""
    if rounds <= 1:
        return np.zeros((0, 2), dtype=np.uint64)
    if samples.size == 0:
        # no data for this reducer: any monotone bounds work
        return np.zeros((rounds - 1, 2), dtype=np.uint64)
    order = np.lexsort((samples[:, 1], samples[:, 0]))
    s = samples[order]
    n = s.shape[0]
    idx = [min(n - 1, (n * q) // rounds) for q in range(1, rounds)]
    return s[idx].astype(np.uint64)


def round_bounds(per_dest_samples: list[np.ndarray], rounds: int) -> np.ndarray:
    """per_dest_samples[d]: (n_d, 2) samples for GPU d (already gathered from all ranks);
    `rounds` = number of cells per GPU.

    Returns a (world, rounds-1, 2) uint64 array."""
    out = [quantile_bounds(s, rounds) for s in per_dest_samples]
    if not out:
        return np.zeros((0, max(rounds - 1, 0), 2), dtype=np.uint64)
    return np.stack(out).astype(np.uint64)
