"""ctypes mirror of the reference's `testcase` (tools/GKL/src/main/native/pairhmm/pairhmm_common.h:20-24)
and helpers to build testcase arrays from PhmmBatch objects (the r-major loop of
benchmarks/phmm/PairHMMUnitTest.cpp:564-579)."""
from __future__ import annotations

import ctypes

import numpy as np


class Testcase(ctypes.Structure):
    _fields_ = [
        ("rslen", ctypes.c_int),
        ("haplen", ctypes.c_int),
        ("q", ctypes.c_void_p),
        ("i", ctypes.c_void_p),
        ("d", ctypes.c_void_p),
        ("c", ctypes.c_void_p),
        ("hap", ctypes.c_void_p),
        ("rs", ctypes.c_void_p),
    ]


TC_DTYPE = np.dtype([("rslen", "<i4"), ("haplen", "<i4"), ("q", "<u8"), ("i", "<u8"), ("d", "<u8"),
                     ("c", "<u8"), ("hap", "<u8"), ("rs", "<u8")])
assert TC_DTYPE.itemsize == ctypes.sizeof(Testcase)


class TestcaseArray:
    """Owns the byte buffers the testcase pointers refer to (the caller owns them in the reference
    too). `arr` is a ctypes array view over a numpy structured buffer (`np_arr`)."""

    __test__ = False  # not a pytest class

    def __init__(self, reads, haps, pairs=None):
        # one contiguous byte pool; every sequence NUL-terminated like strndup
        seqs = []
        for r in reads:
            seqs.extend(r)
        seqs.extend(haps)
        if pairs is not None:
            for rd, h in pairs:
                seqs.extend(rd)
                seqs.append(h)
        lens = np.array([len(s) for s in seqs], np.int64)
        offs = np.zeros(len(seqs) + 1, np.int64)
        np.cumsum(lens + 1, out=offs[1:])
        pool = np.zeros(int(offs[-1]) + 16, np.uint8)
        if seqs:
            pool[np.concatenate([np.arange(o, o + n) for o, n in zip(offs[:-1], lens)])] = \
                np.frombuffer(b"".join(seqs), np.uint8)
        self._pool = pool
        base = pool.ctypes.data
        addr = base + offs[:-1]
        nr, nh = len(reads), len(haps)
        if pairs is None:
            n = nr * nh
            a = np.zeros(max(n, 1), TC_DTYPE)
            if n:
                ra = addr[:5 * nr].reshape(nr, 5)
                rl = lens[:5 * nr].reshape(nr, 5)[:, 0]
                ha = addr[5 * nr:5 * nr + nh]
                hl = lens[5 * nr:5 * nr + nh]
                a["rslen"][:n] = np.repeat(rl, nh)
                a["haplen"][:n] = np.tile(hl, nr)
                for k, f in enumerate(("rs", "q", "i", "d", "c")):
                    a[f][:n] = np.repeat(ra[:, k], nh)
                a["hap"][:n] = np.tile(ha, nr)
        else:
            n = len(pairs)
            a = np.zeros(max(n, 1), TC_DTYPE)
            if n:
                p0 = 5 * nr + nh
                pa = addr[p0:].reshape(n, 6)
                pl = lens[p0:].reshape(n, 6)
                a["rslen"][:n] = pl[:, 0]
                a["haplen"][:n] = pl[:, 5]
                for k, f in enumerate(("rs", "q", "i", "d", "c", "hap")):
                    a[f][:n] = pa[:, k]
        self.n = n
        self.np_arr = a
        self.arr = (Testcase * len(a)).from_address(a.ctypes.data)

    @classmethod
    def from_batch(cls, batch):
        return cls(batch.reads, batch.haps)

    @classmethod
    def from_batches(cls, batches):
        """All batches of a job merged (each batch's r-major cross product, in batch order)."""
        parts = [cls.from_batch(b) for b in batches]
        obj = cls([], [])
        obj._parts = parts
        obj.n = sum(p.n for p in parts)
        a = np.zeros(max(obj.n, 1), TC_DTYPE)
        o = 0
        for p in parts:
            a[o:o + p.n] = p.np_arr[:p.n]
            o += p.n
        obj.np_arr = a
        obj.arr = (Testcase * len(a)).from_address(a.ctypes.data)
        return obj

    @classmethod
    def from_pairs(cls, pairs):
        """pairs: list of (read_tuple, hap_bytes) -> one testcase each (not a cross product)."""
        return cls([], [], pairs=pairs)

    def subset(self, idx):
        """Testcases idx (keeps this object's buffers alive)."""
        obj = TestcaseArray([], [])
        obj._parent = self
        idx = np.asarray(idx)
        obj.n = len(idx)
        a = np.zeros(max(obj.n, 1), TC_DTYPE)
        a[:obj.n] = self.np_arr[idx]
        obj.np_arr = a
        obj.arr = (Testcase * len(a)).from_address(a.ctypes.data)
        return obj

    def cells(self):
        return int((self.np_arr["rslen"][:self.n].astype(np.int64) * self.np_arr["haplen"][:self.n]).sum())
