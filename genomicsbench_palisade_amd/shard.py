"""Work sharding for one process per GPU: every path shards with no exchange --
testcases (phmm), reads (fmi), calls (chain), pairs (bsw). A rank takes a contiguous range of the
work items, balanced by a per-item weight (cells, anchors, ...), so results concatenate in shard
order back into the reference's order."""
from __future__ import annotations

import numpy as np


def balanced_ranges(weights, parts: int):
    """Split items 0..n-1 into `parts` contiguous ranges with near-equal weight sums.

    Boundaries are placed at the item where the running weight crosses k/parts of the total, so
    each range is within one item's weight of the ideal share. Returns [(lo, hi)] (hi exclusive).
    """
    w = np.asarray(weights, dtype=np.float64)
    n = len(w)
    if parts <= 0:
        raise ValueError("parts must be positive")
    if n == 0:
        return [(0, 0)] * parts
    cum = np.cumsum(w)
    total = cum[-1]
    cuts = [0]
    for k in range(1, parts):
        cuts.append(int(np.searchsorted(cum, total * k / parts, side="left")) + 1 if total > 0 else n * k // parts)
    cuts.append(n)
    cuts = np.maximum.accumulate(np.clip(cuts, 0, n))
    return [(int(cuts[k]), int(cuts[k + 1])) for k in range(parts)]


def rank_range(weights, rank: int, world: int):
    """This rank's (lo, hi) of balanced_ranges(weights, world)."""
    return balanced_ranges(weights, world)[rank]
