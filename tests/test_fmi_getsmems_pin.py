"""Pins the oracle's FMI_search::getSMEMs restatement (oracle/fmi_oracle.c) with a second, independent
one: a pure-Python transcription of FMI_search.cpp:1328-1497's control flow over bi-intervals taken
from a brute-force suffix array of the bwa-mem2 index text (forward + reverse complement + '$',
FMI_search.cpp:109-169, :358-434), not from CP_OCC tables. The cases are the ones the reference code
path treats specially: an N met during a forward extension (the smem pushed twice, :1396-1409), an N
met during the backward search (:1426-1431), the in-place prev/curr aliasing (myCurrArray points at
myPrevArray, :1344-1345), the int curr_s (:1422) and the tid-0-only quota when nthreads > 1 (the
OpenMP pragma is commented out, :1340-1351). tests/golden/fmi_getsmems_golden.json holds one case's
expected tuples, written by this file's restatement (make_fixture below) and checked here against
both implementations."""
import json
import os

import numpy as np
import pytest

import fmi_util
from conftest import GOLDEN

FIXTURE = os.path.join(GOLDEN, "fmi_getsmems_golden.json")


class BruteIndex:
    """Bi-intervals (k, l, s) of patterns over the index text, by binary search in a brute-force
    suffix array: k = first row whose suffix starts with P, l = that of revcomp(P), s = count; row 0
    is the '$' suffix (the text's end), as in the bwa-mem2 index (SA[0] = n)."""

    def __init__(self, ref):
        ref = [int(x) for x in ref]
        self.text = ref + [3 - b for b in reversed(ref)]
        n = len(self.text)
        self.sa = sorted(range(n + 1), key=lambda i: self.text[i:] + [-1])
        self.suf = [tuple(self.text[i:]) for i in self.sa]

    def _first(self, p):
        lo, hi = 0, len(self.suf)
        while lo < hi:
            mid = (lo + hi) // 2
            if self.suf[mid] < p:
                lo = mid + 1
            else:
                hi = mid
        return lo

    def interval(self, p):
        p = tuple(p)
        k = self._first(p)
        e = k
        while e < len(self.suf) and self.suf[e][:len(p)] == p:
            e += 1
        rc = tuple(3 - b for b in reversed(p))
        return k, self._first(rc), e - k


def get_smems_py(ix, codes, num_reads, min_seed_len, nthreads):
    """FMI_search::getSMEMs, transcribed (FMI_search.cpp:1328-1497). An SMEM is (rid, m, n, k, l, s)
    plus the pattern it stands for (read[m..n]), whose bi-interval backwardExt / the forward step
    compute here by lookup."""
    rl = codes.shape[1]
    quota = (num_reads + nthreads - 1) // nthreads
    first, last = 0, min(quota, num_reads)  # tid 0 only
    out = []
    for i in range(first, last):
        q = [int(x) for x in codes[i]]
        x = rl - 1
        arr = []  # myPrevArray == myCurrArray
        while x >= 0:
            a = q[x]
            if a > 3:
                x -= 1
                continue
            k, l, s = ix.interval([a])
            smem = dict(rid=i, m=x, n=x, k=k, l=l, s=s)
            num_prev = 0
            arr = []

            def push(e, at):
                if at < len(arr):
                    arr[at] = dict(e)
                else:
                    arr.append(dict(e))
            for j in range(x + 1, rl):
                a = q[j]
                if a < 4:
                    k2, l2, s2 = ix.interval(q[smem["m"]:j + 1])
                    new = dict(smem, k=k2, l=l2, s=s2, n=j)
                    if new["s"] != smem["s"]:
                        push(smem, num_prev)
                        num_prev += 1
                    smem = new
                    if new["s"] == 0:
                        break
                else:
                    push(smem, num_prev)
                    num_prev += 1
                    break
            if smem["s"] != 0:
                push(smem, num_prev)
                num_prev += 1
            arr[:num_prev] = arr[:num_prev][::-1]
            next_x = x - 1
            cur_j = rl
            j = x - 1
            while j >= 0:
                num_curr = 0
                curr_s = -1
                a = q[j]
                if a > 3:
                    next_x = j - 1
                    break
                for p in range(num_prev):
                    sm = arr[p]
                    k2, l2, s2 = ix.interval([a] + q[sm["m"]:sm["n"] + 1])
                    new = dict(sm, k=k2, l=l2, s=s2, m=j)
                    if new["s"] == 0 and num_curr == 0 and j < cur_j:
                        cur_j = j
                        if sm["n"] - sm["m"] + 1 >= min_seed_len:
                            out.append(dict(sm))
                    # curr_s is an int (FMI_search.cpp:1422): compare against the truncated value
                    if new["s"] != 0 and new["s"] != curr_s:
                        curr_s = int(np.int64(new["s"]).astype(np.int32))
                        arr[num_curr] = new
                        num_curr += 1
                num_prev = num_curr
                if num_curr == 0:
                    next_x = j
                    break
                next_x = j - 1
                j -= 1
            if num_prev != 0:
                sm = arr[0]
                if sm["n"] - sm["m"] + 1 >= min_seed_len:
                    out.append(dict(sm))
            x = next_x
    return [(e["rid"], e["m"], e["n"], e["k"], e["l"], e["s"]) for e in out]


def _case(seed, nreads=9, rl=48):
    """A small genome-like reference with repeats, reads from both strands with substitutions, and
    N codes placed inside forward extensions and backward searches."""
    from genomicsbench_palisade_amd import gen
    rng = np.random.default_rng(seed)
    ref = gen.fmi_reference(700, seed=seed, repeat_frac=0.0)
    ref[200:260] = ref[40:100]  # an exact repeat: multi-copy intervals
    ref[400:430] = np.resize(np.array([0, 1], np.uint8), 30)  # a tandem repeat
    codes = np.zeros((nreads, rl), np.uint8)
    for r in range(nreads):
        p = int(rng.integers(0, len(ref) - rl))
        s = ref[p:p + rl].copy()
        if r % 2:
            s = (3 - s[::-1]).astype(np.uint8)
        sub = rng.random(rl) < 0.03
        s[sub] = rng.integers(0, 4, int(sub.sum()), dtype=np.uint8)
        codes[r] = s
    codes[1, rl // 2] = 4          # N in the middle: forward extensions from the right half stop at it
    codes[2, 3] = 4                # N near the start: the backward search stops there
    codes[3, [10, 11, 30]] = 4     # runs of N
    codes[4, rl - 1] = 4           # N at the last base (the first x is skipped)
    codes[5, :] = 4
    codes[5, 20:28] = ref[300:308]  # a read that is almost all N
    return ref, codes


def _oracle(ref, codes, num_reads, min_seed_len, nthreads):
    oi = fmi_util.OracleIndex(ref)
    try:
        got = oi.get_smems(codes, num_reads, min_seed_len, nthreads)
        return [tuple(int(v) for v in (t["rid"], t["m"], t["n"], t["k"], t["l"], t["s"])) for t in got]
    finally:
        oi.close()


def test_brute_intervals_match_oracle_backward_ext():
    """The brute-force bi-intervals agree with the oracle's index on single bases (count[]) -- the
    restatement below and the C oracle share no code, so this checks the row numbering."""
    ref, _ = _case(1)
    ix = BruteIndex(ref)
    oi = fmi_util.OracleIndex(ref)
    n, count5, sentinel = oi.info()
    oi.close()
    assert n == len(ix.sa)
    assert ix.sa.index(0) == sentinel  # the row whose BWT character is '$'
    for a in range(4):
        k, l, s = ix.interval([a])
        assert k == count5[a] and s == count5[a + 1] - count5[a]


@pytest.mark.parametrize("seed,nthreads,min_seed_len", [(1, 1, 12), (2, 3, 10), (3, 2, 15), (4, 1, 6)])
def test_getsmems_oracle_equals_independent_restatement(seed, nthreads, min_seed_len):
    ref, codes = _case(seed)
    exp = get_smems_py(BruteIndex(ref), codes, len(codes), min_seed_len, nthreads)
    assert exp, "the case emits no SMEM"
    got = _oracle(ref, codes, len(codes), min_seed_len, nthreads)
    assert got == exp


def make_fixture():
    ref, codes = _case(2)
    exp = get_smems_py(BruteIndex(ref), codes, len(codes), 10, 3)
    return {"ref": ref.tolist(), "codes": codes.tolist(), "num_reads": len(codes), "min_seed_len": 10,
            "nthreads": 3, "smems": [list(t) for t in exp],
            "note": "FMI_search::getSMEMs (FMI_search.cpp:1328-1497) over this reference and these fixed-stride "
                    "reads (4 = N), tid 0's quota of 3 threads; tuples (rid, m, n, k, l, s) in emission order, "
                    "from tests/test_fmi_getsmems_pin.py's independent restatement (python -c 'import "
                    "test_fmi_getsmems_pin as t, json; json.dump(t.make_fixture(), open(t.FIXTURE, \"w\"))')"}


def test_getsmems_golden_fixture():
    z = json.load(open(FIXTURE))
    ref = np.array(z["ref"], np.uint8)
    codes = np.array(z["codes"], np.uint8)
    exp = [tuple(t) for t in z["smems"]]
    assert get_smems_py(BruteIndex(ref), codes, z["num_reads"], z["min_seed_len"], z["nthreads"]) == exp
    assert _oracle(ref, codes, z["num_reads"], z["min_seed_len"], z["nthreads"]) == exp
    # the fixture covers what it claims: an N inside a read of the processed quota, and a quota
    assert z["nthreads"] > 1 and (codes[:(z["num_reads"] + 2) // 3] == 4).any()
