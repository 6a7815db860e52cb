"""Loaders for the CPU checkers under oracle/ (test infrastructure only)."""
from __future__ import annotations

import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
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
