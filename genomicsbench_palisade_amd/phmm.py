"""Host mirror of the reference PairHMM interface (tools/GKL/src/main/native/pairhmm/
IntelPairHmmCSource.cpp:29-115): init_pairhmm() ~ initPairHMM(), compute_likelihoods_both() ~
computelikelihoodsboth(), all executed by the HIP kernels in libgb.so (csrc/phmm.hip)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import check, lib
from ._tc import Testcase, TestcaseArray  # noqa: F401  (re-exported)


def init_pairhmm():
    check(lib().gb_phmm_init(), "gb_phmm_init")


def compute_likelihoods_both(tcs: TestcaseArray):
    """Returns (results f64, raw_f f32, raw_d f64, used_double u8) for every testcase."""
    n = tcs.n
    res = np.zeros(n, np.float64)
    rf = np.zeros(n, np.float32)
    rd = np.zeros(n, np.float64)
    ud = np.zeros(n, np.uint8)
    if n:
        check(lib().gb_phmm_compute(ctypes.addressof(tcs.arr), n, res.ctypes.data, rf.ctypes.data,
                                    rd.ctypes.data, ud.ctypes.data), "gb_phmm_compute")
    return res, rf, rd, ud


def compute_f64(tcs: TestcaseArray):
    rd = np.zeros(tcs.n, np.float64)
    if tcs.n:
        check(lib().gb_phmm_compute_f64(ctypes.addressof(tcs.arr), tcs.n, rd.ctypes.data),
              "gb_phmm_compute_f64")
    return rd


class DeviceBatch:
    """A packed, HBM-resident testcase batch (gb_phmm_batch_*): create once, run many times."""

    def __init__(self, tcs: TestcaseArray):
        self._tcs = tcs
        self.h = ctypes.c_void_p()
        check(lib().gb_phmm_batch_create(ctypes.addressof(tcs.arr), tcs.n, ctypes.byref(self.h)),
              "gb_phmm_batch_create")

    def run(self):
        check(lib().gb_phmm_batch_run(self.h), "gb_phmm_batch_run")

    def sync(self):
        check(lib().gb_phmm_batch_sync(self.h), "gb_phmm_batch_sync")

    def results(self):
        n = self._tcs.n
        res = np.zeros(n, np.float64)
        rf = np.zeros(n, np.float32)
        rd = np.zeros(n, np.float64)
        ud = np.zeros(n, np.uint8)
        dev = np.zeros(n, np.float64)
        check(lib().gb_phmm_batch_results(self.h, res.ctypes.data, rf.ctypes.data, rd.ctypes.data,
                                          ud.ctypes.data, dev.ctypes.data), "gb_phmm_batch_results")
        return res, rf, rd, ud, dev

    def timing(self):
        a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        check(lib().gb_phmm_batch_timing(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
              "gb_phmm_batch_timing")
        return a.value, b.value, c.value

    def stats(self):
        t, c, f = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(lib().gb_phmm_batch_stats(self.h, ctypes.byref(t), ctypes.byref(c), ctypes.byref(f)),
              "gb_phmm_batch_stats")
        return t.value, c.value, f.value

    def close(self):
        if self.h:
            lib().gb_phmm_batch_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
