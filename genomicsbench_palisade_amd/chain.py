"""Host mirror of the reference chaining interface (host_chain_kernel, benchmarks/chain/src/
host_kernel.cpp:481-501) over CSR call sets (gen.ChainCalls), executed by csrc/chain.hip."""
from __future__ import annotations

import ctypes

import numpy as np

from . import check, lib


def _decl():
    L = lib()
    if getattr(L, "_chain_decl", False):
        return L
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    L.gb_chain_batch_create.argtypes = [i64, vp, vp, vp, vp, vp, ctypes.POINTER(vp)]
    L.gb_chain_batch_run.argtypes = [vp]
    L.gb_chain_batch_sync.argtypes = [vp]
    L.gb_chain_batch_results.argtypes = [vp, vp, vp, vp, vp, vp]
    L.gb_chain_batch_timing.argtypes = [vp, vp]
    L.gb_chain_batch_split_stats.argtypes = [vp, vp, vp, vp]
    L.gb_chain_batch_destroy.argtypes = [vp]
    L.gb_chain_batch_backtrack.argtypes = [vp, ctypes.c_int32, ctypes.c_int32]
    L.gb_chain_batch_chains.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp]
    L.gb_chain_batch_backtrack_timing.argtypes = [vp, vp]
    L._chain_decl = True
    return L


class ChainBatch:
    def __init__(self, calls):
        L = _decl()
        self.calls = calls
        self.h = ctypes.c_void_p()
        check(L.gb_chain_batch_create(calls.ncalls, calls.offsets.ctypes.data, calls.avg_qspan.ctypes.data,
                                      calls.params4.ctypes.data, calls.x.ctypes.data, calls.y.ctypes.data,
                                      ctypes.byref(self.h)), "gb_chain_batch_create")

    def run(self):
        check(_decl().gb_chain_batch_run(self.h), "gb_chain_batch_run")

    def sync(self):
        check(_decl().gb_chain_batch_sync(self.h), "gb_chain_batch_sync")

    def results(self):
        n = self.calls.nanchors
        out = [np.zeros(max(n, 1), np.int32) for _ in range(4)]
        v = ctypes.c_int64()
        check(_decl().gb_chain_batch_results(self.h, *[o.ctypes.data for o in out], ctypes.byref(v)),
              "gb_chain_batch_results")
        return [o[:n] for o in out] + [v.value]

    def timing(self):
        ms = ctypes.c_float()
        check(_decl().gb_chain_batch_timing(self.h, ctypes.byref(ms)), "gb_chain_batch_timing")
        return ms.value

    def split_stats(self):
        """-> (calls run as speculative segments, guess/verify rounds, fix-up blocks) of the last run."""
        v = [ctypes.c_int64() for _ in range(3)]
        check(_decl().gb_chain_batch_split_stats(self.h, *[ctypes.byref(x) for x in v]), "gb_chain_batch_split_stats")
        return tuple(x.value for x in v)

    def backtrack(self, min_cnt: int = 3, min_sc: int = 40):
        """minimap2's chain backtrack on this batch's chain_dp outputs (asynchronous)."""
        check(_decl().gb_chain_batch_backtrack(self.h, min_cnt, min_sc), "gb_chain_batch_backtrack")

    def chains(self):
        """-> (n_chains [ncalls], u [CSR at offsets], n_anchors [ncalls], ax, ay [CSR at 2*offsets],
        total chains, total anchors)."""
        c = self.calls
        n = max(c.nanchors, 1)
        nch = np.zeros(max(c.ncalls, 1), np.int64)
        nan = np.zeros(max(c.ncalls, 1), np.int64)
        u = np.zeros(n, np.uint64)
        ax = np.zeros(2 * n, np.uint64)
        ay = np.zeros(2 * n, np.uint64)
        tc, ta = ctypes.c_int64(), ctypes.c_int64()
        check(_decl().gb_chain_batch_chains(self.h, nch.ctypes.data, u.ctypes.data, nan.ctypes.data, ax.ctypes.data,
                                            ay.ctypes.data, ctypes.byref(tc), ctypes.byref(ta)),
              "gb_chain_batch_chains")
        return nch[:c.ncalls], u, nan[:c.ncalls], ax, ay, tc.value, ta.value

    def backtrack_timing(self):
        ms = ctypes.c_float()
        check(_decl().gb_chain_batch_backtrack_timing(self.h, ctypes.byref(ms)), "gb_chain_batch_backtrack_timing")
        return ms.value

    def close(self):
        if self.h:
            _decl().gb_chain_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
