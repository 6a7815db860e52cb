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


MIN_ACCEPTED = np.float32(1e-28)  # IntelPairHmmCSource.cpp:70: below it the f64 result is used


def compute_f32(tcs: TestcaseArray):
    """computelikelihoodsfloat(): the raw f32 probability of every testcase in full (no early exit)."""
    rf = np.zeros(tcs.n, np.float32)
    if tcs.n:
        check(lib().gb_phmm_compute_f32(ctypes.addressof(tcs.arr), tcs.n, rf.ctypes.data),
              "gb_phmm_compute_f32")
    return rf


def parity_mismatches(got, expect):
    """Mismatch counts of (results, raw_f, raw_d[, used_double]) against the reference's outputs.
    What computelikelihoodsboth exposes is compared bit for bit: the final log10 results, the raw f64
    probabilities and the fallback choice (raw f32 below MIN_ACCEPTED). The raw f32 value is compared
    where the reference's passes MIN_ACCEPTED; where it falls back the f32 pass's early exit may have
    stopped before the last row, so there the device value must be the reference's or exactly 0
    (csrc/phmm.hip phmm_stack kExit)."""
    g_out, g_rf, g_rd = got[:3]
    e_out, e_rf, e_rd = expect[:3]
    passing = e_rf >= MIN_ACCEPTED
    same = g_rf.view(np.uint32) == e_rf.view(np.uint32)
    f32_bad = ~same & (passing | (g_rf.view(np.uint32) != 0))
    return {"log10": int((g_out.view(np.uint64) != e_out.view(np.uint64)).sum()),
            "raw_f32": int(f32_bad.sum()),
            "raw_f64": int((g_rd.view(np.uint64) != e_rd.view(np.uint64)).sum()),
            "f32_dropped": int((~passing & (g_rf == 0) & (e_rf != 0)).sum())}


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

    def exit_stats(self):
        """(testcases the f32 early exit dropped, cells it did not compute) in the last run."""
        d, c = ctypes.c_int64(), ctypes.c_int64()
        check(lib().gb_phmm_batch_exit_stats(self.h, ctypes.byref(d), ctypes.byref(c)),
              "gb_phmm_batch_exit_stats")
        return d.value, c.value

    def close(self):
        if self.h:
            lib().gb_phmm_batch_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
