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
    lib.fmi_oracle_adopt_sa64.argtypes = [vp, i64, vp]
    lib.fmi_oracle_share.argtypes = [vp]
    lib.fmi_oracle_share.restype = vp
    lib.fmi_oracle_unshare.argtypes = [vp]
    lib.fmi_oracle_sa_lookup.argtypes = [vp, vp, i64, ctypes.c_int, vp]
    lib.fmi_oracle_sa_lookup.restype = None
    lib.fmi_oracle_sa_entries.argtypes = [vp, vp, i64, ctypes.c_int32, ctypes.c_int, vp, vp]
    lib.fmi_oracle_sa_entries.restype = i64
    lib.fmi_oracle_lf_steps.argtypes = [vp]
    lib.fmi_oracle_lf_steps.restype = i64
    i32 = ctypes.c_int32
    lib.fmi_oracle_get_smems.argtypes = [vp, vp, i32, i32, i32, i32, vp, vp]
    lib.fmi_oracle_get_smems.restype = None


class OracleIndex:
    def __init__(self, ref_codes=None, path_out=None, load_path=None, adopt=None):
        self.lib = oracle_lib.oracle()
        if not getattr(self.lib, "_fmi_decl", False):
            _decl(self.lib)
            self.lib._fmi_decl = True
        self.h = self.lib.fmi_oracle_new()
        if adopt is not None:  # (n, count5_after_load, sentinel, cp_occ int64[rows, 8][, packed SA])
            n, count5, sentinel, occ = adopt[:4]
            self._occ = np.ascontiguousarray(occ)
            c = np.array([x - 1 for x in count5], np.int64)
            self.lib.fmi_oracle_adopt(self.h, n, c.ctypes.data, sentinel, self._occ.ctypes.data)
            if len(adopt) > 4:
                self._sa = np.ascontiguousarray(adopt[4], np.int64)
                self.lib.fmi_oracle_adopt_sa64(self.h, len(self._sa), self._sa.ctypes.data)
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

    def run_threaded(self, codes, lens, threads, batch_size=512, min_seed_len=19, collect=False):
        """Batches split over `threads` OS threads (ctypes releases the GIL), each with its own
        handle over the shared CP_OCC table; returns (total SMEMs, backwardExt calls), plus with
        collect=True the per-thread SMEM arrays in read order (rid rebased to the whole read set)."""
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
            if collect:
                out = out[:tot].copy()
                out["rid"] += lo
                return tot, calls, out
            return tot, calls

        with ThreadPoolExecutor(threads) as ex:
            res = list(ex.map(work, range(threads)))
        if collect:
            return (sum(r[0] for r in res), sum(r[1] for r in res),
                    [r[2] for r in res if len(r) == 3])
        return sum(r[0] for r in res), sum(r[1] for r in res)

    def bwt_calls(self):
        return self.lib.fmi_oracle_bwt_calls(self.h)

    def sa_lookup(self, rows, mode=0):
        """SA value of each BWT row: mode 0 get_sa_entry_compressed, mode 1 call_one_step chain."""
        rows = np.ascontiguousarray(rows, np.int64)
        out = np.zeros(len(rows), np.int64)
        self.lib.fmi_oracle_sa_lookup(self.h, rows.ctypes.data, len(rows), mode, out.ctypes.data)
        return out

    def sa_entries(self, smems, max_occ=500, mode=1):
        """get_sa_entries(_prefetch) over an SMEM array -> (coords, per-SMEM counts)."""
        smems = np.ascontiguousarray(smems, SMEM_DTYPE)
        cap = int(np.minimum(smems["s"], max_occ).sum()) if len(smems) else 0
        coords = np.zeros(max(cap, 1), np.int64)
        counts = np.zeros(max(len(smems), 1), np.int32)
        tot = self.lib.fmi_oracle_sa_entries(self.h, smems.ctypes.data, len(smems), max_occ, mode,
                                             coords.ctypes.data, counts.ctypes.data)
        assert tot == cap
        return coords[:tot], counts[:len(smems)]

    def get_smems(self, codes, num_reads, min_seed_len=19, nthreads=1):
        """FMI_search::getSMEMs restated (fixed-stride reads of codes.shape[1] bases) -> SMEM array."""
        codes = np.ascontiguousarray(codes, np.uint8)
        rl = codes.shape[1]
        out = np.zeros(max(1, num_reads * (rl + 2) * 2), SMEM_DTYPE)
        tot = np.zeros(max(1, nthreads), np.int64)
        self.lib.fmi_oracle_get_smems(self.h, codes.ctypes.data, num_reads, rl, min_seed_len, nthreads,
                                      out.ctypes.data, tot.ctypes.data)
        return out[:tot[0]]

    def lf_steps(self):
        return self.lib.fmi_oracle_lf_steps(self.h)

    def sa_entries_threaded(self, smems, threads, max_occ=500, mode=1):
        """sa_entries over `threads` OS threads (shared tables); returns (coordinates, LF steps)."""
        from concurrent.futures import ThreadPoolExecutor
        smems = np.ascontiguousarray(smems, SMEM_DTYPE)
        parts = np.array_split(np.arange(len(smems)), threads)

        def work(ix):
            if len(ix) == 0:
                return 0, 0
            sub = np.ascontiguousarray(smems[ix[0]:ix[-1] + 1])
            h = self.lib.fmi_oracle_share(self.h)
            cap = int(np.minimum(np.maximum(sub["s"], 0), max_occ).sum())
            coords = np.zeros(max(cap, 1), np.int64)
            tot = self.lib.fmi_oracle_sa_entries(h, sub.ctypes.data, len(sub), max_occ, mode,
                                                 coords.ctypes.data, None)
            steps = self.lib.fmi_oracle_lf_steps(h)
            self.lib.fmi_oracle_unshare(h)
            return tot, steps

        with ThreadPoolExecutor(threads) as ex:
            res = list(ex.map(work, parts))
        return sum(r[0] for r in res), sum(r[1] for r in res)

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
    lib.ref_bwa_sa.argtypes = [vp, ctypes.c_char_p, vp, i64, vp]
    lib.ref_bwa_from_cp_occ.argtypes = [vp, i64, i64]
    lib.ref_bwa_from_cp_occ.restype = vp
    lib.ref_bwa_collect_batch.argtypes = [vp, vp, vp, i64, i64, ctypes.c_int]
    lib.ref_bwa_collect_batch.restype = i64
    return lib


def bwa_from_tables(lib, n, sentinel, cp_occ):
    """bwa v1 bwt_t over the BWT held by bwa-mem2 CP_OCC tables (same row numbering)."""
    cp = np.ascontiguousarray(cp_occ, np.int64)
    return lib.ref_bwa_from_cp_occ(cp.ctypes.data, n, sentinel)


def bwa_collect_threaded(lib, bwt, codes, lens, threads, min_seed_len=19):
    """bwa v1 mem_collect_intv over every read, reads split over `threads` OS threads (ctypes
    releases the GIL); returns the total interval count."""
    from concurrent.futures import ThreadPoolExecutor
    codes = np.ascontiguousarray(codes, np.uint8)
    lens = np.ascontiguousarray(lens, np.int32)
    parts = np.array_split(np.arange(len(lens)), threads)

    def work(ix):
        if len(ix) == 0:
            return 0
        lo, hi = int(ix[0]), int(ix[-1]) + 1
        return lib.ref_bwa_collect_batch(bwt, codes[lo:hi].ctypes.data, lens[lo:hi].ctypes.data, hi - lo,
                                         codes.shape[1], min_seed_len)
    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(work, parts))
    assert min(res) >= 0
    return int(sum(res))


def bwa_sa(lib, bwt, sa_path, rows):
    """bwa v1 bwt_sa (tools/bwa/bwt.c:86) over its own .sa file."""
    rows = np.ascontiguousarray(rows, np.int64)
    out = np.zeros(len(rows), np.int64)
    assert lib.ref_bwa_sa(bwt, sa_path.encode(), rows.ctypes.data, len(rows), out.ctypes.data) == 0
    return out


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


# ------------------------------------------------------------------ index structure (any size)
def bwt_char(cp_occ, rows):
    """BWT byte at each row from the CP_OCC one-hot words (bit 63 - (row & 63) of line row >> 6,
    build_fm_index FMI_search.cpp:290-320); 4 where no base bit is set (the sentinel row)."""
    rows = np.asarray(rows, np.int64)
    line = cp_occ[rows >> 6]
    bit = np.uint64(63) - (rows & 63).astype(np.uint64)
    out = np.full(len(rows), 4, np.int64)
    for b in range(4):
        hit = ((line[:, 4 + b].view(np.uint64) >> bit) & np.uint64(1)).astype(bool)
        out[hit] = b
    return out


def suffix_less(text, a, b, window=64):
    """Vectorised lexicographic suffix comparison text[a:] < text[b:] with end-of-text smallest (the
    order saisxx gives the reference's build, FMI_search.cpp:250). Returns a bool array."""
    a = np.asarray(a, np.int64).copy()
    b = np.asarray(b, np.int64).copy()
    n = len(text)
    res = np.zeros(len(a), bool)
    todo = np.arange(len(a))
    pad = np.concatenate([text.astype(np.int16), np.full(window, -1, np.int16)])
    while len(todo):
        ia, ib = a[todo], b[todo]
        wa = pad[np.minimum(ia[:, None] + np.arange(window)[None, :], n + window - 1)]
        wb = pad[np.minimum(ib[:, None] + np.arange(window)[None, :], n + window - 1)]
        wa[ia[:, None] + np.arange(window)[None, :] >= n] = -1
        wb[ib[:, None] + np.arange(window)[None, :] >= n] = -1
        diff = wa != wb
        anyd = diff.any(axis=1)
        first = diff.argmax(axis=1)
        r = np.arange(len(todo))
        res[todo[anyd]] = wa[r[anyd], first[anyd]] < wb[r[anyd], first[anyd]]
        # equal windows that ran into the end of text: the shorter suffix is smaller
        ended = (~anyd) & ((ia + window >= n) | (ib + window >= n))
        res[todo[ended]] = ia[ended] > ib[ended]
        todo = todo[(~anyd) & ~ended]
        a[todo] += window
        b[todo] += window
    return res


def check_index_structure(ref, n, count5, sentinel, cp_occ, sa_sampled=None, sample=20000, seed=0):
    """Size-independent invariants of a .bwt.2bit.64 index over text = ref + revcomp(ref) (+ '$'):
    CP_OCC counts are the running popcounts of the one-hot words, every row holds exactly one base
    except the sentinel, per-base totals equal the text's base counts, and -- on the sampled SA --
    the sampled rows are distinct, in suffix order, and carry BWT[row] = text[SA[row] - 1]. Raises
    AssertionError with the first violated invariant."""
    text = np.concatenate([ref, (3 - ref[::-1]).astype(np.uint8)])
    assert n == len(text) + 1
    rows_total = (n >> 6) + 1
    assert cp_occ.shape == (rows_total, 8)
    oh = cp_occ[:, 4:].view(np.uint64)
    cnt = cp_occ[:, :4]
    pc = np.bitwise_count(oh).astype(np.int64)
    assert (cnt[1:] == cnt[:-1] + pc[:-1]).all(), "cp_count is not the running popcount"
    assert (cnt[0] == 0).all()
    for i in range(4):
        for j in range(i + 1, 4):
            assert not (oh[:, i] & oh[:, j]).any(), "a BWT row carries two bases"
    per_line = pc.sum(axis=1)
    full = np.full(rows_total, 64, np.int64)
    full[-1] = n - (rows_total - 1) * 64
    full[sentinel >> 6] -= 1
    assert (per_line == full).all(), "rows without a base other than the sentinel"
    assert bwt_char(cp_occ, [sentinel])[0] == 4
    c4 = np.bincount(text, minlength=4)[:4].astype(np.int64)
    assert ((cnt[-1] + pc[-1]) == c4).all(), "per-base totals differ from the text"
    exp5 = np.concatenate([[0], np.cumsum(c4)]) + 1
    assert list(count5) == exp5.tolist(), (count5, exp5)
    if sa_sampled is None:
        return
    ns = (n >> 3) + 1
    sa = np.asarray(sa_sampled, np.int64)[:ns]
    assert sa.min() >= 0 and sa.max() < n
    seen = np.zeros(n, np.uint8)
    seen[sa] = 1
    assert int(seen.sum(dtype=np.int64)) == len(sa), "sampled SA entries repeat"
    del seen
    rng = np.random.default_rng(seed)
    t = np.unique(rng.integers(0, ns, sample))
    rows = t * 8
    s = sa[t]
    exp = np.where(s > 0, text[np.maximum(s - 1, 0)], 4)
    assert (bwt_char(cp_occ, rows) == exp).all(), "BWT[row] != text[SA[row] - 1]"
    t2 = t[t + 1 < ns]
    assert suffix_less(text, sa[t2], sa[t2 + 1]).all(), "sampled SA rows out of suffix order"


def read_index_file(path):
    """(n, count5 as stored, cp_occ int64[rows, 8], packed sampled SA int64, sentinel) of a
    .bwt.2bit.64 file (layout of build_fm_index, FMI_search.cpp:171-356)."""
    raw = np.fromfile(path, np.uint8)
    n = int(raw[:8].view(np.int64)[0])
    count5 = raw[8:48].view(np.int64).copy()
    sz = (n >> 6) + 1
    o = 48
    cp = raw[o:o + sz * 64].view(np.int64).reshape(sz, 8)
    o += sz * 64
    ns = (n >> 3) + 1
    ms = raw[o:o + ns].view(np.int8).astype(np.int64)
    ls = raw[o + ns:o + 5 * ns].view(np.uint32).astype(np.int64)
    sentinel = int(raw[o + 5 * ns:o + 5 * ns + 8].view(np.int64)[0])
    return n, count5, cp, (ms << 32) | ls, sentinel


def call_one_step(n_count5_loaded, cp, sa, pos, offset=0):
    """call_one_step (FMI_search.cpp:1834-1893) restated over the file tables: (ret, sa_entry, offset)."""
    if pos & 7 == 0:
        return 1, int(sa[pos >> 3]), offset
    line = cp[pos >> 6]
    y = 63 - (pos & 63)
    b = 4
    for c in range(4):
        if (int(line[4 + c]) >> y) & 1:
            b = c
            break
    if b == 4:
        return 1, 0, offset
    yy = pos & 63
    mask = ((1 << 64) - 1) ^ ((1 << (64 - yy)) - 1) if yy else 0
    occ = int(line[b]) + bin((int(line[4 + b]) & ((1 << 64) - 1)) & mask).count("1")
    sp = int(n_count5_loaded[b]) + occ
    offset += 1
    if sp & 7 == 0:
        return 1, int(sa[sp >> 3]) + offset, offset
    return 0, sp, offset
