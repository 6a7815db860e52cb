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


# ---- the per-path shards bench.py (strong scaling) and tests/test_dist.py take -----------------
FMI_BATCH = 512  # fmi.cpp batch size: shards hold whole batches so per-batch outputs do not change


def testcase_range(tcs, rank: int, world: int):
    """phmm: contiguous testcases balanced by cells (rslen * haplen)."""
    a = tcs.np_arr[:tcs.n]
    return rank_range(a["rslen"].astype(np.int64) * a["haplen"], rank, world)


def shard_testcases(tcs, rank: int, world: int):
    lo, hi = testcase_range(tcs, rank, world)
    return tcs.subset(np.arange(lo, hi)), (lo, hi)


def read_range(nreads: int, rank: int, world: int, batch: int = FMI_BATCH):
    """fmi: contiguous whole batches of reads, equal batch counts (reads are equal-length)."""
    nb = (nreads + batch - 1) // batch
    lo, hi = rank_range(np.ones(nb), rank, world)
    return min(lo * batch, nreads), min(hi * batch, nreads)


def call_range(calls, rank: int, world: int):
    """chain: contiguous calls balanced by anchor count."""
    return rank_range(np.diff(calls.offsets), rank, world)


def shard_calls(calls, rank: int, world: int):
    lo, hi = call_range(calls, rank, world)
    return calls.slice(lo, hi), (lo, hi)


def pair_range(pairs, rank: int, world: int):
    """bsw: contiguous pairs balanced by the band-cell estimate qlen * tlen."""
    return rank_range(pairs.qlen.astype(np.int64) * pairs.tlen, rank, world)


def shard_pairs(pairs, rank: int, world: int):
    lo, hi = pair_range(pairs, rank, world)
    return pairs.slice(lo, hi), (lo, hi)
