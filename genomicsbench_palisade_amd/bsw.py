"""Host mirror of the reference banded-SW interface (BandedPairWiseSW::getScores16 over SeqPair,
benchmarks/bsw/bandedSWA.h:92-101,120-124,195-200), executed by csrc/bsw.hip.

Pairs are gen.BswPairs (flattened target/query buffers, SeqPair.idr/idq = offsets into them).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import check, lib

# SeqPair (bandedSWA.h:92-101) == gb_seqpair (include/gb_bsw.h), 72 bytes
SEQPAIR_DTYPE = np.dtype([("idr", "<i8"), ("idq", "<i8"), ("id", "<i8"), ("len1", "<i4"), ("len2", "<i4"),
                          ("h0", "<i4"), ("seqid", "<i4"), ("regid", "<i4"), ("score", "<i4"), ("tle", "<i4"),
                          ("gtle", "<i4"), ("qle", "<i4"), ("gscore", "<i4"), ("max_off", "<i4"),
                          ("_pad", "<i4")])
assert SEQPAIR_DTYPE.itemsize == 72

# out6 order used by the C ABI, the oracle and the reference shim
OUT_FIELDS = ("score", "qle", "tle", "gtle", "gscore", "max_off")


class Params(ctypes.Structure):
    """gb_bsw_params: BandedPairWiseSW constructor arguments + getScores16's w."""
    _fields_ = [("o_del", ctypes.c_int32), ("e_del", ctypes.c_int32), ("o_ins", ctypes.c_int32),
                ("e_ins", ctypes.c_int32), ("zdrop", ctypes.c_int32), ("end_bonus", ctypes.c_int32),
                ("w", ctypes.c_int32), ("mat", ctypes.c_int8 * 25)]

    def as_array(self):
        """{o_del, e_del, o_ins, e_ins, zdrop, end_bonus, w} as the oracle takes them."""
        return np.array([self.o_del, self.e_del, self.o_ins, self.e_ins, self.zdrop, self.end_bonus, self.w],
                        np.int32)

    def mat_array(self):
        return np.array(list(self.mat), np.int8)


def fill_scmat(a=1, b=4, ambig=-1):
    """bwa_fill_scmat (main_banded.cpp:77-88)."""
    m = np.full((5, 5), ambig, np.int8)
    for i in range(4):
        for j in range(4):
            m[i, j] = a if i == j else -b
    return m.reshape(-1)


def default_params(**kw):
    """The benchmark's settings (main_banded.cpp:53-57,846): 1/4/-1, gaps 6+1, zdrop 100, end_bonus 5, w 100."""
    p = Params(6, 1, 6, 1, 100, 5, 100)
    mat = kw.pop("mat", None)
    if mat is None:
        mat = fill_scmat(kw.pop("match", 1), kw.pop("mismatch", 4), kw.pop("ambig", -1))
    for k, v in kw.items():
        setattr(p, k, int(v))
    for k in range(25):
        p.mat[k] = int(mat[k])
    return p


def seqpairs(pairs):
    """SeqPair records for a BswPairs set, ids batch-local like loadPairs (main_banded.cpp:177-197)."""
    sp = np.zeros(pairs.n, SEQPAIR_DTYPE)
    sp["idr"], sp["idq"], sp["id"] = pairs.toff, pairs.qoff, np.arange(pairs.n)
    sp["len1"], sp["len2"], sp["h0"] = pairs.tlen, pairs.qlen, pairs.h0
    for f in ("seqid", "regid", "score", "tle", "gtle", "qle", "gscore", "max_off"):
        sp[f] = -1
    return sp


def _decl():
    L = lib()
    if getattr(L, "_bsw_decl", False):
        return L
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    L.gb_bsw_batch_create.argtypes = [vp, vp, i64, vp, i64, vp, i64, ctypes.POINTER(vp)]
    L.gb_bsw_batch_run.argtypes = [vp]
    L.gb_bsw_batch_sync.argtypes = [vp]
    L.gb_bsw_batch_results.argtypes = [vp, vp, vp, vp, vp]
    L.gb_bsw_batch_timing.argtypes = [vp, vp]
    L.gb_bsw_batch_destroy.argtypes = [vp]
    L.gb_bsw_get_scores16.argtypes = [vp, vp, i64, vp, i64, vp, i64]
    L.gb_bsw_default_params.argtypes = [vp]
    L._bsw_decl = True
    return L


def _buf(a):
    return a.ctypes.data if len(a) else None


class BswBatch:
    """Pairs resident on the current device; run() extends them all (one kernel launch)."""

    def __init__(self, pairs, params=None):
        L = _decl()
        self.pairs = pairs
        self.params = params if params is not None else default_params()
        self._sp = seqpairs(pairs)
        self.h = ctypes.c_void_p()
        check(L.gb_bsw_batch_create(ctypes.byref(self.params), _buf(self._sp), pairs.n, _buf(pairs.tgt),
                                    len(pairs.tgt), _buf(pairs.qry), len(pairs.qry), ctypes.byref(self.h)),
              "gb_bsw_batch_create")

    def run(self):
        check(_decl().gb_bsw_batch_run(self.h), "gb_bsw_batch_run")

    def sync(self):
        check(_decl().gb_bsw_batch_sync(self.h), "gb_bsw_batch_sync")

    def results(self, want_cells=True):
        """(out6 int32 [n,6] = score,qle,tle,gtle,gscore,max_off; cells int32 [n] or None; total cells)."""
        n = self.pairs.n
        out6 = np.zeros((max(n, 1), 6), np.int32)
        cells = np.zeros(max(n, 1), np.int32) if want_cells else None
        tot = ctypes.c_int64()
        check(_decl().gb_bsw_batch_results(self.h, None, out6.ctypes.data,
                                           cells.ctypes.data if want_cells else None, ctypes.byref(tot)),
              "gb_bsw_batch_results")
        return out6[:n], (cells[:n] if want_cells else None), tot.value

    def timing(self):
        ms = ctypes.c_float()
        check(_decl().gb_bsw_batch_timing(self.h, ctypes.byref(ms)), "gb_bsw_batch_timing")
        return ms.value

    def close(self):
        if self.h:
            _decl().gb_bsw_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def get_scores16(pairs, params=None):
    """One-shot getScores16: returns the SeqPair array with score/tle/gtle/qle/gscore/max_off filled."""
    params = params if params is not None else default_params()
    sp = seqpairs(pairs)
    check(_decl().gb_bsw_get_scores16(ctypes.byref(params), _buf(sp), pairs.n, _buf(pairs.tgt), len(pairs.tgt),
                                      _buf(pairs.qry), len(pairs.qry)), "gb_bsw_get_scores16")
    return sp


def get_scores8(pairs, params=None, w_match: int = 1):
    """One-shot getScores8 (the 8-bit path's domain only: len1, len2 < 128, h0 + min(len1, len2) *
    w_match < 128, bwamem.cpp:2152-2155; raises GbError for any other pair)."""
    params = params if params is not None else default_params()
    sp = seqpairs(pairs)
    L = _decl()
    L.gb_bsw_get_scores8.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                     ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    check(L.gb_bsw_get_scores8(ctypes.byref(params), w_match, _buf(sp), pairs.n, _buf(pairs.tgt), len(pairs.tgt),
                               _buf(pairs.qry), len(pairs.qry), None), "gb_bsw_get_scores8")
    return sp
