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


def batch_bounds(tcs):
    """Testcase offsets of the job's batches (TestcaseArray.from_batches keeps its parts), or the
    whole job as one batch."""
    parts = getattr(tcs, "_parts", None)
    if not parts:
        return np.array([0, tcs.n], np.int64)
    return np.concatenate([[0], np.cumsum([p.n for p in parts])]).astype(np.int64)


def testcase_index(tcs, rank: int, world: int):
    """phmm, stratified: the rank's piece of EVERY batch -- each batch's testcases cut into `world`
    contiguous pieces balanced by cells. Batches differ in how many testcases fall back to the f64
    pass (36 % of the 'large' job overall, 31-41 % across contiguous 1/8 shards), so contiguous
    shards of whole batches differ in cost by more than their cells; a piece of every batch carries
    the job's mix. Returns the rank's testcase indices, ascending (the union over ranks is every
    testcase once; results gather back by these indices)."""
    a = tcs.np_arr[:tcs.n]
    w = a["rslen"].astype(np.int64) * a["haplen"]
    b = batch_bounds(tcs)
    idx = []
    for b0, b1 in zip(b[:-1], b[1:]):
        lo, hi = rank_range(w[b0:b1], rank, world)
        idx.append(np.arange(b0 + lo, b0 + hi, dtype=np.int64))
    return np.concatenate(idx) if idx else np.zeros(0, np.int64)


def shard_testcases(tcs, rank: int, world: int):
    """-> (the rank's testcases, their indices in the job)."""
    idx = testcase_index(tcs, rank, world)
    return tcs.subset(idx), idx


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


# ---- output digests: a rank's shard outputs against a 1-rank pass, without moving the outputs ------
# Each output unit (a testcase's result, an anchor's chain_dp outputs, an SMEM at its place in its
# batch, a pair's six fields) hashes together with its GLOBAL key (testcase index, anchor index,
# (batch, position in batch), pair index); a set's digest is the sum of its units' hashes mod 2^64. The
# sum does not depend on how the units are split over ranks, and the keys make it order-sensitive, so
# sum(rank digests) == digest(1-rank pass) iff every unit landed where the 1-rank pass puts it (up to a
# 2^-64 collision). bench.py gathers one (digest, units) pair per leg and rank.
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def mix64(x):
    """splitmix64's finaliser over a uint64 array (wrapping arithmetic)."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * _M1
        x = (x ^ (x >> np.uint64(27))) * _M2
        return x ^ (x >> np.uint64(31))


def _as_u64(c):
    c = np.asarray(c)
    if c.dtype.kind == "f":
        c = c.view(np.uint64 if c.itemsize == 8 else np.uint32)
    return c.astype(np.int64).view(np.uint64) if c.dtype.kind == "i" else c.astype(np.uint64)


def unit_hashes(keys, *cols):
    """Per-unit 64-bit hashes of (key, col0[i], col1[i], ...); floats hash by their bits."""
    with np.errstate(over="ignore"):
        h = (_as_u64(keys) ^ _GOLD) * _M1
        for c in cols:  # xor-multiply-shift per column (4 array ops), one full finaliser at the end
            h ^= _as_u64(c)
            h *= _M2
            h ^= h >> np.uint64(29)
        return mix64(h)


def digest(keys, *cols) -> int:
    """sum(unit_hashes) mod 2^64 as a Python int (0 for no units)."""
    if len(keys) == 0:
        return 0
    return int(np.add.reduce(unit_hashes(keys, *cols), dtype=np.uint64))


def digest_add(*ds) -> int:
    return sum(int(d) for d in ds) % (1 << 64)


def smem_keys(rid, batch_counts, first_batch: int):
    """fmi: the global key of each SMEM of a shard's output -- (global batch, position inside the batch)
    -- from the per-batch counts of the shard (its batches are whole, the first one `first_batch`)."""
    bc = np.asarray(batch_counts, np.int64)
    starts = np.repeat(np.cumsum(bc) - bc, bc)
    pos = np.arange(len(starts), dtype=np.int64) - starts
    b = np.repeat(np.arange(first_batch, first_batch + len(bc), dtype=np.int64), bc)
    if len(rid) != len(pos):
        raise ValueError("SMEM count does not match the per-batch counts")
    return (b << 32) | pos
