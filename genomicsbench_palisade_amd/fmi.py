"""Host mirror of the reference FMI_search interface (tools/bwa-mem2/src/FMI_search.h:101-224) and
the fmi benchmark pipeline (benchmarks/fmi/fmi.cpp:253-348), executed by the HIP kernels in
libgb.so (csrc/fmi.hip, csrc/fmi_build.hip, csrc/fmi_sa.hip). SA lookup: get_sa_entry_compressed /
get_sa_entries_prefetch (FMI_search.cpp:1714-2040)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import check, lib

SA_COMPRESSED = 0  # get_sa_entry_compressed (FMI_search.cpp:1714-1807)
SA_PREFETCH = 1    # get_sa_entries_prefetch / call_one_step (:1834-2040), what bwamem.cpp:737 calls
MAX_OCC = 500      # bwa-mem2's default opt->max_occ

SMEM_DTYPE = np.dtype([("rid", "<u4"), ("m", "<u4"), ("n", "<u4"), ("pad", "<u4"),
                       ("k", "<i8"), ("l", "<i8"), ("s", "<i8")])  # == SMEM (FMI_search.h:91-99)


def _decl():
    L = lib()
    if getattr(L, "_fmi_decl", False):
        return L
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
    L.gb_fmi_index_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
    L.gb_fmi_index_build.argtypes = [vp, i64, ctypes.c_char_p, ctypes.POINTER(vp)]
    L.gb_fmi_index_info.argtypes = [vp, vp, vp, vp]
    L.gb_fmi_index_cp_occ.argtypes = [vp, vp, i64]
    L.gb_fmi_index_destroy.argtypes = [vp]
    L.gb_fmi_reads_create.argtypes = [vp, vp, vp, i32, i32, ctypes.POINTER(vp)]
    L.gb_fmi_reads_destroy.argtypes = [vp]
    L.gb_fmi_search.argtypes = [vp, i32]
    L.gb_fmi_debug_ctl.argtypes = [vp, vp]
    L.gb_fmi_get_smems.argtypes = [vp, vp, i32, i32, i32, i32, vp, i64, vp, vp]
    L.gb_fmi_sync.argtypes = [vp]
    L.gb_fmi_results.argtypes = [vp, i32, vp, i64, vp, vp, vp]
    L.gb_fmi_timing.argtypes = [vp, vp, vp, vp]
    L.gb_fmi_index_sa.argtypes = [vp, vp, i64]
    L.gb_fmi_sa_lookup.argtypes = [vp, vp, i64, i32, vp]
    L.gb_fmi_sa_entries.argtypes = [vp, vp, i64, i32, i32, vp, i64, vp, vp]
    L.gb_fmi_reads_sa_run.argtypes = [vp, i32, i32]
    L.gb_fmi_reads_sa_results.argtypes = [vp, vp, i64, vp, vp]
    L.gb_fmi_reads_sa_timing.argtypes = [vp, vp, vp, vp]
    L._fmi_decl = True
    return L


class Index:
    """FMI_search(prefix) + load_index() (or build_index()) with the index resident in HBM."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def load(cls, path: str):
        L = _decl()
        h = ctypes.c_void_p()
        check(L.gb_fmi_index_load(path.encode(), ctypes.byref(h)), "gb_fmi_index_load")
        return cls(h)

    @classmethod
    def build(cls, ref_codes: np.ndarray, out_path: str | None = None):
        L = _decl()
        ref = np.ascontiguousarray(ref_codes, np.uint8)
        h = ctypes.c_void_p()
        check(L.gb_fmi_index_build(ref.ctypes.data, len(ref), out_path.encode() if out_path else None,
                                   ctypes.byref(h)), "gb_fmi_index_build")
        return cls(h)

    def info(self):
        n, s = ctypes.c_int64(), ctypes.c_int64()
        c = (ctypes.c_int64 * 5)()
        check(_decl().gb_fmi_index_info(self.h, ctypes.byref(n), c, ctypes.byref(s)), "gb_fmi_index_info")
        return n.value, list(c), s.value

    def cp_occ(self):
        n, _, _ = self.info()
        size = (n >> 6) + 1
        buf = np.zeros(size * 8, np.int64)
        check(_decl().gb_fmi_index_cp_occ(self.h, buf.ctypes.data, buf.nbytes), "gb_fmi_index_cp_occ")
        return buf.reshape(size, 8)

    def sampled_sa(self):
        n, _, _ = self.info()
        buf = np.zeros((n >> 3) + 1, np.int64)
        check(_decl().gb_fmi_index_sa(self.h, buf.ctypes.data, len(buf)), "gb_fmi_index_sa")
        return buf

    def sa_lookup(self, rows, mode: int = SA_PREFETCH) -> np.ndarray:
        """SA value of each BWT row (one LF walk per row on the GPU)."""
        rows = np.ascontiguousarray(rows, np.int64)
        out = np.zeros(max(len(rows), 1), np.int64)
        check(_decl().gb_fmi_sa_lookup(self.h, rows.ctypes.data, len(rows), mode, out.ctypes.data),
              "gb_fmi_sa_lookup")
        return out[:len(rows)]

    def sa_entries(self, smems, max_occ: int = MAX_OCC, mode: int = SA_PREFETCH):
        """get_sa_entries(_prefetch) over an SMEM array -> (coords, per-SMEM counts)."""
        smems = np.ascontiguousarray(smems, SMEM_DTYPE)
        n = len(smems)
        cap = int(np.minimum(np.maximum(smems["s"], 0), max_occ).sum()) if n else 0
        coords = np.zeros(max(cap, 1), np.int64)
        counts = np.zeros(max(n, 1), np.int32)
        tot = ctypes.c_int64()
        check(_decl().gb_fmi_sa_entries(self.h, smems.ctypes.data, n, max_occ, mode, coords.ctypes.data,
                                        len(coords), counts.ctypes.data, ctypes.byref(tot)),
              "gb_fmi_sa_entries")
        return coords[:tot.value], counts[:n]

    def get_smems(self, codes: np.ndarray, num_reads: int, min_seed_len: int = 19, nthreads: int = 1):
        """FMI_search::getSMEMs over fixed-stride reads (codes: num_reads x readlength) -> (SMEMs in the
        reference's order, backwardExt calls)."""
        L = _decl()
        codes = np.ascontiguousarray(codes, np.uint8)
        rl = codes.shape[1] if codes.ndim == 2 else 0
        n, calls = ctypes.c_int64(), ctypes.c_int64()
        check(L.gb_fmi_get_smems(self.h, codes.ctypes.data, num_reads, rl, min_seed_len, nthreads, None, 0,
                                 ctypes.byref(n), ctypes.byref(calls)), "gb_fmi_get_smems")
        out = np.zeros(max(n.value, 1), SMEM_DTYPE)
        check(L.gb_fmi_get_smems(self.h, codes.ctypes.data, num_reads, rl, min_seed_len, nthreads, out.ctypes.data,
                                 len(out), ctypes.byref(n), ctypes.byref(calls)), "gb_fmi_get_smems")
        return out[:n.value], calls.value

    def close(self):
        if self.h:
            _decl().gb_fmi_index_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Reads:
    """enc_qdb (numReads x max_readlength codes) + lengths resident in HBM, searched many times."""

    def __init__(self, index: Index, codes: np.ndarray, lens: np.ndarray):
        L = _decl()
        self.index = index
        self.codes = np.ascontiguousarray(codes, np.uint8)
        self.lens = np.ascontiguousarray(lens, np.int32)
        self.n, self.maxlen = self.codes.shape
        self.h = ctypes.c_void_p()
        check(L.gb_fmi_reads_create(index.h, self.codes.ctypes.data, self.lens.ctypes.data, self.n,
                                    self.maxlen, ctypes.byref(self.h)), "gb_fmi_reads_create")

    def search(self, min_seed_len: int = 19):
        check(_decl().gb_fmi_search(self.h, min_seed_len), "gb_fmi_search")

    def sync(self):
        check(_decl().gb_fmi_sync(self.h), "gb_fmi_sync")

    def results(self, batch_size: int = 512, want_smems: bool = True):
        L = _decl()
        tot = ctypes.c_int64()
        nb = (self.n + batch_size - 1) // batch_size
        bc = np.zeros(max(nb, 1), np.int64)
        pc = np.zeros(3, np.int64)
        check(L.gb_fmi_results(self.h, batch_size, None, 0, ctypes.byref(tot), bc.ctypes.data,
                               pc.ctypes.data), "gb_fmi_results")
        out = None
        if want_smems:
            out = np.zeros(max(tot.value, 1), SMEM_DTYPE)
            check(L.gb_fmi_results(self.h, batch_size, out.ctypes.data, len(out), None, None, None),
                  "gb_fmi_results")
            out = out[:tot.value]
        return out, tot.value, bc[:nb], pc

    def timing(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        c = ctypes.c_int64()
        check(_decl().gb_fmi_timing(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
              "gb_fmi_timing")
        return a.value, b.value, c.value

    def ctl(self):
        """The last search's control words (gb_fmi_debug_ctl): reads taken, big slots taken, fatal
        overflows, 0, reads handed to the wave pass."""
        out = np.zeros(8, np.int32)
        check(_decl().gb_fmi_debug_ctl(self.h, out.ctypes.data), "gb_fmi_debug_ctl")
        return out

    def sa_run(self, max_occ: int = MAX_OCC, mode: int = SA_PREFETCH):
        """SA coordinates of the last search's SMEMs, on the device (bwamem.cpp:737 for every read)."""
        check(_decl().gb_fmi_reads_sa_run(self.h, max_occ, mode), "gb_fmi_reads_sa_run")

    def sa_results(self, want_coords: bool = True):
        L = _decl()
        tot = ctypes.c_int64()
        check(L.gb_fmi_reads_sa_results(self.h, None, 0, None, ctypes.byref(tot)), "gb_fmi_reads_sa_results")
        if not want_coords:
            return None, None, tot.value
        coords = np.zeros(max(tot.value, 1), np.int64)
        _, ns, _, _ = self.results(want_smems=False)
        counts = np.zeros(max(ns, 1), np.int32)
        check(L.gb_fmi_reads_sa_results(self.h, coords.ctypes.data, len(coords), counts.ctypes.data, None),
              "gb_fmi_reads_sa_results")
        return coords[:tot.value], counts[:ns], tot.value

    def sa_timing(self):
        """(kernel ms, LF steps, coordinates) of the last sa_run."""
        a = ctypes.c_float()
        st, nc = ctypes.c_int64(), ctypes.c_int64()
        check(_decl().gb_fmi_reads_sa_timing(self.h, ctypes.byref(a), ctypes.byref(st), ctypes.byref(nc)),
              "gb_fmi_reads_sa_timing")
        return a.value, st.value, nc.value

    def close(self):
        if self.h:
            _decl().gb_fmi_reads_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
