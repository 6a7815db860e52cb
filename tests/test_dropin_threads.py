"""GPU: the one-shot drop-in entry points (gb_phmm_compute = computelikelihoodsboth, gb_bsw_get_scores16
= BandedPairWiseSW::getScores16) called concurrently from several host threads, the way the
reference's OpenMP teams call them (bsw: main_banded.cpp:896-909, one object per thread). Each
thread reuses its own cached device workspace across calls; results must stay bit-exact against
the oracle. Also the PairHMM haplotype-length cap (kMaxHaplen, csrc/phmm.hip): lengths up to it
are bit-exact, longer ones are rejected with GB_ERR_ARG instead of faulting."""
import ctypes
import threading

import numpy as np
import pytest

import oracle_lib
from conftest import assert_phmm_exact, bits
from genomicsbench_palisade_amd import gen
from genomicsbench_palisade_amd._tc import TestcaseArray

MAX_HAPLEN = 65535  # csrc/phmm.hip kMaxHaplen (longer than kLdsHaplen = 9400: records in global scratch)


def _phmm_oracle(ta):
    o = oracle_lib.oracle()
    out, rf, rd = np.zeros(ta.n), np.zeros(ta.n, np.float32), np.zeros(ta.n)
    o.phmm_oracle_batch(ctypes.addressof(ta.arr), ta.n, out.ctypes.data, rf.ctypes.data, rd.ctypes.data, None, 8)
    return out, rf, rd


def _run_threads(fn, n):
    errs, res = [], [None] * n

    def work(k):
        try:
            res[k] = fn(k)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=work, args=(k,)) for k in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    return res


@pytest.mark.gpu
def test_phmm_compute_threads_reuse_workspaces():
    from genomicsbench_palisade_amd import phmm, set_device
    set_device(0)
    phmm.init_pairhmm()
    rng = np.random.default_rng(17)
    jobs = [TestcaseArray.from_batch(gen.phmm_batch(rng, int(rng.integers(2, 12)), int(rng.integers(1, 6))))
            for _ in range(12)]
    exp = [_phmm_oracle(t) for t in jobs]

    def fn(k):
        from genomicsbench_palisade_amd import set_device as sd
        sd(0)
        out = []
        for rep in range(3):  # several calls per thread: the cached batch is refilled (grow + shrink)
            for j in range(k, len(jobs), 4):
                out.append((j, phmm.compute_likelihoods_both(jobs[j])))
        return out

    for res in _run_threads(fn, 4):
        for j, got in res:
            assert_phmm_exact(got, exp[j])


@pytest.mark.gpu
def test_bsw_get_scores16_threads():
    from genomicsbench_palisade_amd import bsw, set_device
    set_device(0)
    params = bsw.default_params()
    sets = [gen.bsw_pairs(int(n), seed=100 + k) for k, n in enumerate((512, 300, 512, 77, 512, 512, 1, 400))]
    exp = [oracle_lib.bsw_oracle(p, params, 4)[0] for p in sets]

    def fn(k):
        from genomicsbench_palisade_amd import set_device as sd
        sd(0)
        out = []
        for rep in range(2):
            for j in range(k, len(sets), 4):
                sp = bsw.get_scores16(sets[j], params)
                out.append((j, np.stack([sp["score"], sp["qle"], sp["tle"], sp["gtle"], sp["gscore"],
                                         sp["max_off"]], axis=1)))
        return out

    for res in _run_threads(fn, 4):
        for j, got in res:
            assert (got == exp[j]).all(), j


@pytest.mark.gpu
def test_phmm_long_haplotypes_up_to_the_cap():
    from genomicsbench_palisade_amd import phmm, set_device
    set_device(0)
    phmm.init_pairhmm()
    rng = np.random.default_rng(5)
    pairs = []
    for hl in (4097, 9400, 9401, 20000):
        for rl in (1, 64, 65, 130):
            hap = rng.choice(np.frombuffer(b"ACGT", np.uint8), hl)
            st = int(rng.integers(0, hl - rl + 1))
            rd = hap[st:st + rl].copy()
            q = rng.integers(6, 41, rl).astype(np.uint8)
            i = rng.integers(40, 46, rl).astype(np.uint8)
            d = rng.integers(40, 46, rl).astype(np.uint8)
            c = np.full(rl, 10, np.uint8)
            pairs.append(((rd.tobytes(), q.tobytes(), i.tobytes(), d.tobytes(), c.tobytes()), hap.tobytes()))
    ta = TestcaseArray.from_pairs(pairs)
    got = phmm.compute_likelihoods_both(ta)
    exp = _phmm_oracle(ta)
    assert_phmm_exact(got, exp)
    # device-resident batch path too (f32 + persistent f64 grid)
    b = phmm.DeviceBatch(ta)
    b.run()
    r = b.results()
    assert (bits(r[0]) == bits(exp[0])).all()
    b.close()


@pytest.mark.gpu
def test_phmm_over_cap_rejected():
    from genomicsbench_palisade_amd import GbError, phmm, set_device
    set_device(0)
    phmm.init_pairhmm()
    hap = b"ACGT" * ((MAX_HAPLEN + 4) // 4)
    rd = b"ACGTACGTAC"
    qs = bytes([30] * 10), bytes([45] * 10), bytes([45] * 10), bytes([10] * 10)
    ta = TestcaseArray.from_pairs([((rd,) + qs, hap[:MAX_HAPLEN + 1])])
    with pytest.raises(GbError):
        phmm.compute_likelihoods_both(ta)
