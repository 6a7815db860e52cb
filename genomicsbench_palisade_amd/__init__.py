"""genomicsbench_palisade_amd -- MI355X-native (gfx950) drop-in for GenomicsBench's hot kernels.

The product is the C-ABI library lib/libgb.so (hand-written HIP for gfx950, declared in
include/gb_*.h) plus the reference-compatible drop-ins (lib/libgkl_pairhmm_c.so, bin/phmm).
This package is the thin Python host mirror used by tests and bench.py: it loads the in-tree
libgb.so with ctypes and fails loudly if it is missing -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
LIB_DIR = os.path.join(PKG_DIR, "lib")
LIBGB = os.path.join(LIB_DIR, "libgb.so")

_lib = None


class GbError(RuntimeError):
    pass


def lib():
    """The loaded libgb.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIBGB):
            raise GbError(f"{LIBGB} not built: run `make` (or __graft_entry__.build()) first")
        _lib = ctypes.CDLL(LIBGB)
        _declare(_lib)
    return _lib


def _declare(L):
    vp, ci, i64p = ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)
    fp = ctypes.POINTER(ctypes.c_float)
    L.gb_last_error.restype = ctypes.c_char_p
    L.gb_device_count.argtypes = [ctypes.POINTER(ci)]
    L.gb_set_device.argtypes = [ci]
    L.gb_phmm_init.argtypes = []
    L.gb_phmm_compute.argtypes = [vp, ci, vp, vp, vp, vp]
    L.gb_phmm_compute_f64.argtypes = [vp, ci, vp]
    L.gb_phmm_compute_f32.argtypes = [vp, ci, vp]
    L.gb_phmm_batch_create.argtypes = [vp, ci, ctypes.POINTER(vp)]
    L.gb_phmm_batch_run.argtypes = [vp]
    L.gb_phmm_batch_sync.argtypes = [vp]
    L.gb_phmm_batch_results.argtypes = [vp, vp, vp, vp, vp, vp]
    L.gb_phmm_batch_timing.argtypes = [vp, fp, fp, fp]
    L.gb_phmm_batch_stats.argtypes = [vp, i64p, i64p, i64p]
    L.gb_phmm_batch_exit_stats.argtypes = [vp, i64p, i64p]
    L.gb_phmm_batch_destroy.argtypes = [vp]


def check(status: int, what: str = "gb call"):
    if status != 0:
        msg = lib().gb_last_error().decode(errors="replace")
        raise GbError(f"{what} failed ({status}): {msg}")


def device_count() -> int:
    n = ctypes.c_int(0)
    st = lib().gb_device_count(ctypes.byref(n))
    return n.value if st == 0 else 0


def set_device(dev: int):
    check(lib().gb_set_device(dev), "gb_set_device")
