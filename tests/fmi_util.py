"""Test helpers for the fmi path: oracle handles, reference (bwa v1) cross-check, fixtures."""
from __future__ import annotations

import ctypes
import os

import numpy as np

import oracle_lib

SMEM_DTYPE = np.dtype([("rid", "<u4"), ("m", "<u4"), ("n", "<u4"), ("pad", "<u4"),
                       ("k", "<i8"), ("l", "<i8"), ("s", "<i8")])
assert SMEM_DTYPE.itemsize == 40


def _decl(lib):
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    lib.fmi_oracle_new.restype = vp
    lib.fmi_oracle_delete.argtypes = [vp]
    lib.fmi_oracle_build.argtypes = [vp, i64, ctypes.c_char_p, vp]
    lib.fmi_oracle_load.argtypes = [ctypes.c_char_p, vp]
    lib.fmi_oracle_run.argtypes = [vp, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_int32, vp, i64, vp, vp]
    lib.fmi_oracle_run.restype = i64
    lib.fmi_oracle_bwt_calls.argtypes = [vp]
    lib.fmi_oracle_bwt_calls.restype = i64
    lib.fmi_oracle_info.argtypes = [vp, vp, vp, vp]
    lib.fmi_oracle_adopt.argtypes = [vp, i64, vp, i64, vp]
    lib.fmi_oracle_share.argtypes = [vp]
    lib.fmi_oracle_share.restype = vp
    lib.fmi_oracle_unshare.argtypes = [vp]


class OracleIndex:
    def __init__(self, ref_codes=None, path_out=None, load_path=None, adopt=None):
        self.lib = oracle_lib.oracle()
        if not getattr(self.lib, "_fmi_decl", False):
            _decl(self.lib)
            self.lib._fmi_decl = True
        self.h = self.lib.fmi_oracle_new()
        if adopt is not None:  # (n, count5_after_load, sentinel, cp_occ int64[rows, 8])
            n, count5, sentinel, occ = adopt
            self._occ = np.ascontiguousarray(occ)
            c = np.array([x - 1 for x in count5], np.int64)
            self.lib.fmi_oracle_adopt(self.h, n, c.ctypes.data, sentinel, self._occ.ctypes.data)
            self._adopted = True
            return
        if load_path is not None:
            st = self.lib.fmi_oracle_load(load_path.encode(), self.h)
        else:
            ref = np.ascontiguousarray(ref_codes, np.uint8)
            st = self.lib.fmi_oracle_build(ref.ctypes.data, len(ref),
                                           path_out.encode() if path_out else None, self.h)
        assert st == 0, st

    def info(self):
        n = ctypes.c_int64()
        c = (ctypes.c_int64 * 5)()
        s = ctypes.c_int64()
        self.lib.fmi_oracle_info(self.h, ctypes.byref(n), c, ctypes.byref(s))
        return n.value, list(c), s.value

    def run(self, codes, lens, batch_size=512, min_seed_len=19):
        codes = np.ascontiguousarray(codes, np.uint8)
        lens = np.ascontiguousarray(lens, np.int32)
        nreads, maxlen = codes.shape
        cap = nreads * (8 * maxlen + 64)
        out = np.zeros(cap, SMEM_DTYPE)
        nb = (nreads + batch_size - 1) // batch_size
        bc = np.zeros(nb, np.int64)
        pc = np.zeros(3, np.int64)
        tot = self.lib.fmi_oracle_run(self.h, codes.ctypes.data, lens.ctypes.data, nreads, maxlen,
                                      batch_size, min_seed_len, out.ctypes.data, cap,
                                      bc.ctypes.data, pc.ctypes.data)
        assert tot >= 0
        return out[:tot], bc, pc

    def run_threaded(self, codes, lens, threads, batch_size=512, min_seed_len=19):
        """Batches split over `threads` OS threads (ctypes releases the GIL), each with its own
        handle over the shared CP_OCC table; returns (total SMEMs, backwardExt calls)."""
        from concurrent.futures import ThreadPoolExecutor
        codes = np.ascontiguousarray(codes, np.uint8)
        lens = np.ascontiguousarray(lens, np.int32)
        nreads, maxlen = codes.shape
        nb = (nreads + batch_size - 1) // batch_size
        per = (nb + threads - 1) // threads * batch_size

        def work(t):
            lo, hi = t * per, min(nreads, (t + 1) * per)
            if lo >= hi:
                return 0, 0
            h = self.lib.fmi_oracle_share(self.h)
            cap = (hi - lo) * (8 * maxlen + 64)
            out = np.zeros(cap, SMEM_DTYPE)
            tot = self.lib.fmi_oracle_run(h, codes[lo:hi].ctypes.data, lens[lo:hi].ctypes.data, hi - lo,
                                          maxlen, batch_size, min_seed_len, out.ctypes.data, cap, None, None)
            calls = self.lib.fmi_oracle_bwt_calls(h)
            self.lib.fmi_oracle_unshare(h)
            return tot, calls

        with ThreadPoolExecutor(threads) as ex:
            res = list(ex.map(work, range(threads)))
        return sum(r[0] for r in res), sum(r[1] for r in res)

    def bwt_calls(self):
        return self.lib.fmi_oracle_bwt_calls(self.h)

    def close(self):
        if self.h:
            if getattr(self, "_adopted", False):
                self.lib.fmi_oracle_unshare(self.h)  # tables belong to self._occ
            else:
                self.lib.fmi_oracle_delete(self.h)
            self.h = None


def ref_bwa():
    path = os.path.join(oracle_lib.ROOT, "oracle", "_ref", "libref_bwa.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    lib.ref_bwa_build.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.ref_bwa_load.argtypes = [ctypes.c_char_p]
    lib.ref_bwa_load.restype = vp
    lib.ref_bwa_free.argtypes = [vp]
    lib.ref_bwa_collect.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp, i64]
    lib.ref_bwa_collect.restype = i64
    return lib


def bwa_smems(lib, bwt, codes, lens, min_seed_len=19):
    """Per read: sorted list of (m, n, k, l, s) from bwa v1's mem_collect_intv."""
    out = []
    cap = 4096
    k, l, s = (np.zeros(cap, np.int64) for _ in range(3))
    m, n = np.zeros(cap, np.int32), np.zeros(cap, np.int32)
    for r in range(len(lens)):
        q = np.ascontiguousarray(codes[r, :lens[r]], np.uint8)
        c = lib.ref_bwa_collect(bwt, q.ctypes.data, int(lens[r]), min_seed_len, k.ctypes.data,
                                l.ctypes.data, s.ctypes.data, m.ctypes.data, n.ctypes.data, cap)
        assert c >= 0
        out.append(sorted(zip(m[:c].tolist(), n[:c].tolist(), k[:c].tolist(), l[:c].tolist(),
                              s[:c].tolist())))
    return out


def per_read(smems, nreads):
    """Group an SMEM array by rid -> sorted list of (m, n, k, l, s)."""
    out = [[] for _ in range(nreads)]
    for r, m, n, k, l, s in zip(smems["rid"], smems["m"], smems["n"], smems["k"], smems["l"], smems["s"]):
        out[int(r)].append((int(m), int(n), int(k), int(l), int(s)))
    return [sorted(x) for x in out]
