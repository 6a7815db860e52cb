"""Loaders for the CPU checkers under oracle/ (test infrastructure only)."""
from __future__ import annotations

import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# GB_ORACLE_SO selects another build of the same sources (tools/sanitize.sh: ASan + UBSan)
ORACLE_SO = os.environ.get("GB_ORACLE_SO") or os.path.join(ROOT, "oracle", "_build", "liboracle.so")
REF_PHMM_SO = os.path.join(ROOT, "oracle", "_ref", "libref_phmm.so")

_oracle = None
_ref = None


def oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"])
        lib = ctypes.CDLL(ORACLE_SO)
        vp = ctypes.c_void_p
        lib.phmm_oracle_batch.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, ctypes.c_int]
        lib.phmm_oracle_batch.restype = None
        lib.phmm_oracle_prob_f32.argtypes = [vp]
        lib.phmm_oracle_prob_f32.restype = ctypes.c_float
        lib.phmm_oracle_prob_f64.argtypes = [vp]
        lib.phmm_oracle_prob_f64.restype = ctypes.c_double
        lib.phmm_oracle_init()
        _oracle = lib
    return _oracle


def ref_phmm():
    """The reference's own GKL kernels (oracle/_ref); None when not built."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_PHMM_SO):
            return None
        lib = ctypes.CDLL(REF_PHMM_SO)
        vp = ctypes.c_void_p
        lib.ref_phmm_batch.argtypes = [vp, ctypes.c_int, vp, vp, vp, ctypes.c_int, ctypes.c_int]
        lib.ref_phmm_batch.restype = None
        lib.ref_phmm_has_avx512.restype = ctypes.c_int
        _ref = lib
    return _ref


def _chain_decl(lib, fn):
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    getattr(lib, fn).argtypes = [i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int]


def chain_oracle(calls, nthreads=4):
    """oracle/chain_oracle.c over a gen.ChainCalls -> (scores, parents, targets, peaks, visited)."""
    import numpy as np
    lib = oracle()
    if not getattr(lib, "_chain_decl", False):
        _chain_decl(lib, "chain_oracle_batch")
        lib.chain_oracle_batch.restype = ctypes.c_int64
        lib._chain_decl = True
    n = calls.nanchors
    out = [np.zeros(max(n, 1), np.int32) for _ in range(4)]
    visited = lib.chain_oracle_batch(calls.ncalls, calls.offsets.ctypes.data, calls.avg_qspan.ctypes.data,
                                     calls.params4.ctypes.data, calls.x.ctypes.data, calls.y.ctypes.data,
                                     *[o.ctypes.data for o in out], nthreads)
    return [o[:n] for o in out] + [visited]


def ref_chain():
    path = os.path.join(ROOT, "oracle", "_ref", "libref_chain.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    _chain_decl(lib, "ref_chain_batch")
    lib.ref_chain_batch.restype = None
    return lib


def ref_chain_run(lib, calls, nthreads=4):
    import numpy as np
    n = calls.nanchors
    out = [np.zeros(max(n, 1), np.int32) for _ in range(4)]
    lib.ref_chain_batch(calls.ncalls, calls.offsets.ctypes.data, calls.avg_qspan.ctypes.data,
                        calls.params4.ctypes.data, calls.x.ctypes.data, calls.y.ctypes.data,
                        *[o.ctypes.data for o in out], nthreads)
    return [o[:n] for o in out]


def _bsw_args(pairs, params):
    import numpy as np
    mat = np.ascontiguousarray(params.mat_array())
    par = np.ascontiguousarray(params.as_array())
    tgt = pairs.tgt if len(pairs.tgt) else np.zeros(1, np.uint8)
    qry = pairs.qry if len(pairs.qry) else np.zeros(1, np.uint8)
    keep = (mat, par, tgt, qry)
    return keep, [pairs.n, tgt.ctypes.data, pairs.toff.ctypes.data, pairs.tlen.ctypes.data, qry.ctypes.data,
                  pairs.qoff.ctypes.data, pairs.qlen.ctypes.data, pairs.h0.ctypes.data, mat.ctypes.data,
                  par.ctypes.data]


def bsw_oracle(pairs, params, nthreads=4):
    """oracle/bsw_oracle.c over gen.BswPairs -> (out6 [n,6], cells [n], total cells)."""
    import numpy as np
    lib = oracle()
    if not getattr(lib, "_bsw_decl", False):
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        lib.bsw_oracle_batch.argtypes = [i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int]
        lib.bsw_oracle_batch.restype = ctypes.c_int64
        lib._bsw_decl = True
    out = np.zeros((max(pairs.n, 1), 6), np.int32)
    cells = np.zeros(max(pairs.n, 1), np.int64)
    keep, a = _bsw_args(pairs, params)
    tot = lib.bsw_oracle_batch(*a, out.ctypes.data, cells.ctypes.data, nthreads)
    return out[:pairs.n], cells[:pairs.n], tot


def ref_bsw():
    """bwa v1 ksw_extend2 compiled from the reference tree (oracle/_ref/libref_bwa.so) or None."""
    path = os.path.join(ROOT, "oracle", "_ref", "libref_bwa.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    lib.ref_bwa_ksw_batch.argtypes = [i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.ref_bwa_ksw_batch.restype = None
    return lib


def ref_bsw_run(lib, pairs, params):
    import numpy as np
    out = np.zeros((max(pairs.n, 1), 6), np.int32)
    keep, a = _bsw_args(pairs, params)
    lib.ref_bwa_ksw_batch(*a, out.ctypes.data)
    return out[:pairs.n]


def chain_bt_oracle(calls, f, p, v, min_cnt=3, min_sc=40, nthreads=4):
    """oracle/chain_oracle.c chain_oracle_backtrack_batch -> (n_chains [ncalls], u list, (bx, by) list)
    per call, from chain_dp outputs f (scores), p (parents), v (peak scores)."""
    import numpy as np
    lib = oracle()
    if not getattr(lib, "_chain_bt_decl", False):
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        lib.chain_oracle_backtrack_batch.argtypes = [i64, vp, vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int,
                                                     vp, vp, vp, vp, vp, ctypes.c_int]
        lib.chain_oracle_backtrack_batch.restype = None
        lib._chain_bt_decl = True
    n = max(calls.nanchors, 1)
    f, p, v = (np.ascontiguousarray(a, np.int32) for a in (f, p, v))
    u = np.zeros(n, np.uint64)
    bx = np.zeros(2 * n, np.uint64)
    by = np.zeros(2 * n, np.uint64)
    nch = np.zeros(max(calls.ncalls, 1), np.int64)
    nan = np.zeros(max(calls.ncalls, 1), np.int64)
    lib.chain_oracle_backtrack_batch(calls.ncalls, calls.offsets.ctypes.data, f.ctypes.data, p.ctypes.data,
                                     v.ctypes.data, calls.x.ctypes.data, calls.y.ctypes.data, min_cnt, min_sc,
                                     u.ctypes.data, bx.ctypes.data, by.ctypes.data, nch.ctypes.data,
                                     nan.ctypes.data, nthreads)
    return unpack_chain_bt(calls.offsets, calls.ncalls, nch, nan, u, bx, by)


def unpack_chain_bt(offsets, ncalls, nch, nan, u, bx, by):
    """CSR backtrack outputs (u at offsets[c], anchors at 2*offsets[c]) -> per-call lists."""
    us, anchors = [], []
    for c in range(ncalls):
        o = int(offsets[c])
        us.append(u[o:o + int(nch[c])].copy())
        anchors.append((bx[2 * o:2 * o + int(nan[c])].copy(), by[2 * o:2 * o + int(nan[c])].copy()))
    return nch[:ncalls].copy(), us, anchors


def ref_chain_bt():
    """The minimap2-acceleration testbed mm_chain_dp (DP + backtrack) compiled from the reference
    tree (oracle/_ref/libref_chain_bt.so) or None."""
    path = os.path.join(ROOT, "oracle", "_ref", "libref_chain_bt.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.ref_chain_dp_bt.argtypes = [i64, ci, ci, ci, ci, ci, ci, ci, vp, vp, vp, vp, vp, vp]
    lib.ref_chain_dp_bt.restype = i64
    return lib


def ref_chain_bt_run(lib, calls, min_cnt=3, min_sc=40, max_skip=25):
    """Per call: (u, (bx, by)) from the reference mm_chain_dp. The reference computes avg_qspan from
    the anchors (testbed/chain.c:40-41); callers compare on calls whose avg_qspan field equals that."""
    import numpy as np
    us, anchors = [], []
    for c in range(calls.ncalls):
        o0, o1 = int(calls.offsets[c]), int(calls.offsets[c + 1])
        n = o1 - o0
        x = np.ascontiguousarray(calls.x[o0:o1])
        y = np.ascontiguousarray(calls.y[o0:o1])
        u = np.zeros(max(n, 1), np.uint64)
        bx = np.zeros(2 * max(n, 1), np.uint64)
        by = np.zeros(2 * max(n, 1), np.uint64)
        na = ctypes.c_int64()
        p4 = np.asarray(calls.params4).reshape(-1)[4 * c:4 * c + 4]
        k = lib.ref_chain_dp_bt(n, int(p4[0]), int(p4[1]), int(p4[2]), max_skip, min_cnt, min_sc, int(p4[3]),
                                x.ctypes.data, y.ctypes.data, u.ctypes.data, bx.ctypes.data, by.ctypes.data,
                                ctypes.byref(na))
        us.append(u[:k].copy())
        anchors.append((bx[:na.value].copy(), by[:na.value].copy()))
    return us, anchors
