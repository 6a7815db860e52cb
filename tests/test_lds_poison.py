"""Stale-LDS guard (GPU): every CU's LDS is first filled with an adversarial pattern
(tests/cpp/lds_poison.hip: all ones, word index + 1, small constants that equal an "i + 1" stamp of
an early anchor, hashed words), then the LDS-heavy kernels run on inputs whose outputs depend on their
LDS words -- chain_rows + verify_lanes (stamp rings, the split path), smem_search (the LDS `prev` head
and staged read codes), bsw_lane_kernel (query codes), phmm_forward (a stack's boundary records and
haplotype codes, both passes; the two-row kernel; the f32 early exit) and the FMI_search class
methods' per-call kernels (fmi_task_wave's per-launch LDS lists and codes) -- and must stay
oracle-exact. A kernel that reads
a word it did not write in its own workgroup (chain_rows' stamps before commit 1da81ef) fails here
deterministically instead of once in a while."""
import ctypes
import os

import numpy as np
import pytest

import fmi_util
import oracle_lib
from conftest import ROOT
from genomicsbench_palisade_amd import gen

pytestmark = pytest.mark.gpu

# (mode, value): 0 all ones, 1 word + 1, 2 constant, 3 word + constant, 4 hashed
PATTERNS = [(0, 0), (1, 0), (2, 2), (2, 37), (2, 300), (3, 1000), (4, 0)]


@pytest.fixture(scope="module")
def poison():
    path = os.path.join(ROOT, "tests", "_build", "liblds_poison.so")
    if not os.path.exists(path):
        pytest.fail(f"{path} not built (make)")
    lib = ctypes.CDLL(path)
    lib.lds_poison.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
    from genomicsbench_palisade_amd import set_device
    set_device(0)

    def run(mode, value, seed=1):
        st = lib.lds_poison(0, mode, value, seed)
        assert st == 0, f"lds_poison failed: hip error {st}"
    return run


CHAIN_NAMES = ["scores", "parents", "targets", "peak_scores"]


@pytest.mark.parametrize("vlanes", ["1", "0"])
def test_chain_after_poison(poison, monkeypatch, vlanes):
    """chain_rows (two calls per wave, stamp rings) and the speculative split path (verify_lanes, or
    verify_kernel alone with GB_CHAIN_VLANES=0) on calls long enough to be split into segments."""
    from genomicsbench_palisade_amd import chain
    monkeypatch.setenv("GB_CHAIN_VLANES", vlanes)
    calls = gen.chain_dataset("small", num_calls=400, seed=21, median_n=1500, max_n=40000)
    exp = oracle_lib.chain_oracle(calls, 8)
    b = chain.ChainBatch(calls)
    try:
        for mode, value in PATTERNS:
            poison(mode, value)
            b.run()
            got = b.results()
            for k, name in enumerate(CHAIN_NAMES):
                bad = np.nonzero(got[k] != exp[k])[0]
                assert len(bad) == 0, f"pattern {(mode, value)}: {name} differs at {len(bad)} anchors, first {bad[:5]}"
            assert got[4] == exp[4], f"pattern {(mode, value)}: visited {got[4]} vs {exp[4]}"
            assert b.split_stats()[0] > 0  # the split path ran
    finally:
        b.close()


def test_fmi_search_after_poison(poison, tmp_path):
    from genomicsbench_palisade_amd import fmi
    ref = gen.fmi_reference(300_000, seed=31)
    codes, lens = gen.fmi_reads(ref, 6000, read_len=151, seed=131, sub_rate=0.02, n_rate=0.002)
    p = str(tmp_path / "r.bwt.2bit.64")
    oi = fmi_util.OracleIndex(ref, path_out=p)
    exp, ebc, epc = oi.run(codes, lens, batch_size=512)
    idx = fmi.Index.load(p)
    rs = fmi.Reads(idx, codes, lens)
    try:
        for mode, value in PATTERNS:
            poison(mode, value)
            rs.search(19)
            sm, tot, bc, pc = rs.results(batch_size=512)
            assert tot == len(exp) and (bc == ebc).all() and (pc == epc).all(), f"pattern {(mode, value)}"
            for f in ("rid", "m", "n", "k", "l", "s"):
                assert (sm[f] == exp[f]).all(), f"pattern {(mode, value)}: field {f}"
            assert rs.timing()[2] == oi.bwt_calls()
    finally:
        rs.close()
        idx.close()
        oi.close()


@pytest.mark.parametrize("tail", ["0", "1"])
def test_bsw_after_poison(poison, monkeypatch, tail):
    """tail "0": the pair-per-lane kernels (bsw_lane_kernel's LDS query codes and per-lane constants),
    "1": the wave-per-pair kernel."""
    from genomicsbench_palisade_amd import bsw
    monkeypatch.setenv("GB_BSW_TAIL", tail)
    p = gen.bsw_pairs(30000, seed=41)
    P = bsw.default_params()
    exp, ocells, _ = oracle_lib.bsw_oracle(p, P, nthreads=8)
    b = bsw.BswBatch(p, P)
    try:
        for mode, value in PATTERNS:
            poison(mode, value)
            b.run()
            got, cells, _ = b.results()
            bad = np.nonzero((got[:p.n] != exp[:p.n]).any(axis=1))[0]
            assert len(bad) == 0, f"pattern {(mode, value)}: {len(bad)} pairs differ, first {bad[:5]}"
            assert (cells[:p.n] == ocells[:p.n]).all()
    finally:
        b.close()


@pytest.mark.parametrize("knob", ["", "GB_PHMM_RPL=2", "GB_PHMM_EXIT=0"])
def test_phmm_after_poison(poison, monkeypatch, knob):
    """phmm_forward<float> (default: with the early exit; the two-row kernel; without the exit) and the
    f64 fallback's persistent grid, on a job with partial stripes and both passes."""
    import ctypes as ct
    from conftest import assert_phmm_exact
    from genomicsbench_palisade_amd import phmm, set_device
    from genomicsbench_palisade_amd._tc import TestcaseArray
    if knob:
        k, v = knob.split("=")
        monkeypatch.setenv(k, v)
    set_device(0)
    phmm.init_pairhmm()
    rng = np.random.default_rng(19)
    ta = TestcaseArray.from_batches([gen.phmm_batch(rng, 40, 16) for _ in range(3)])
    o = oracle_lib.oracle()
    exp = np.zeros(ta.n), np.zeros(ta.n, np.float32), np.zeros(ta.n)
    o.phmm_oracle_batch(ct.addressof(ta.arr), ta.n, exp[0].ctypes.data, exp[1].ctypes.data, exp[2].ctypes.data,
                        None, 8)
    assert (exp[1] < 1e-28).any()
    b = phmm.DeviceBatch(ta)
    try:
        for mode, value in PATTERNS:
            poison(mode, value)
            b.run()
            got = b.results()
            assert_phmm_exact(got[:4], exp)
    finally:
        b.close()


def test_fmi_class_tasks_after_poison(poison):
    """The FMI_search class methods' per-call kernels (getSMEMsAllPosOneThread, getSMEMsOnePosOneThread,
    bwtSeedStrategyAllPosOneThread: fmi_task_wave with its per-launch dynamic LDS) give the same
    records after every poison pattern as before any, and AllPos + LAST give the batched search's
    (oracle-exact) SMEM sets per read."""
    import ctypes as ct
    from genomicsbench_palisade_amd import fmi, lib
    L = lib()
    vp, i32, i64 = ct.c_void_p, ct.c_int32, ct.c_int64
    L.gb_fmi_smem_allpos.argtypes = [vp, vp, vp, vp, i32, vp, vp, i32, i32, vp, i64, vp, vp, vp]
    L.gb_fmi_smem_onepos.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp, i32, i32, vp, i64, vp, vp, vp]
    L.gb_fmi_last_seeds.argtypes = [vp, vp, vp, vp, i32, vp, i32, vp, i64, vp, vp]
    ref = gen.fmi_reference(300_000, seed=33, repeat_frac=0.2)
    codes, lens = gen.fmi_reads(ref, 600, read_len=151, seed=133, sub_rate=0.03, n_rate=0.002)
    n = len(lens)
    flat = np.ascontiguousarray(codes[:, :151]).reshape(-1).astype(np.uint8)
    offs = (np.arange(n, dtype=np.int32) * 151).astype(np.int32)
    lens32 = lens.astype(np.int32)
    rid = np.arange(n, dtype=np.int32)
    ones = np.ones(n, np.int32)
    twenty = np.full(n, 20, np.int32)
    qpos = (np.arange(n) % 100).astype(np.int16)
    idx = fmi.Index.build(ref)
    cap = 200 * n

    def call():
        outs = []
        for which in ("allpos", "onepos", "last"):
            out = np.zeros(cap, fmi_util.SMEM_DTYPE)
            nout, calls = ct.c_int64(), ct.c_int64()
            if which == "allpos":
                st = L.gb_fmi_smem_allpos(idx.h, flat.ctypes.data, lens32.ctypes.data, offs.ctypes.data, n,
                                          ones.ctypes.data, rid.ctypes.data, n, 19, out.ctypes.data, cap,
                                          ct.byref(nout), None, ct.byref(calls))
            elif which == "onepos":
                nxt = np.zeros(n, np.int16)
                st = L.gb_fmi_smem_onepos(idx.h, flat.ctypes.data, lens32.ctypes.data, offs.ctypes.data, n,
                                          qpos.ctypes.data, ones.ctypes.data, rid.ctypes.data, n, 19,
                                          out.ctypes.data, cap, ct.byref(nout), nxt.ctypes.data, ct.byref(calls))
            else:
                st = L.gb_fmi_last_seeds(idx.h, flat.ctypes.data, lens32.ctypes.data, offs.ctypes.data, n,
                                         twenty.ctypes.data, 20, out.ctypes.data, cap, ct.byref(nout), ct.byref(calls))
            assert st == 0, (which, L.gb_last_error())
            outs.append((out[:nout.value].copy(), calls.value))
        return outs

    try:
        clean = call()
        assert all(len(o) > 0 for o, _ in clean)
        for mode, value in PATTERNS:
            poison(mode, value)
            got = call()
            for (a, ca), (b, cb) in zip(got, clean):
                assert ca == cb and len(a) == len(b), f"pattern {(mode, value)}"
                for f in ("rid", "m", "n", "k", "l", "s"):
                    assert (a[f] == b[f]).all(), f"pattern {(mode, value)}: field {f}"
        # AllPos (min_intv 1) + LAST (max_intv 20, min length 20) = phases 1 and 3 of the batched search
        oi = fmi_util.OracleIndex(ref)
        exp, _, epc = oi.run(codes, lens, batch_size=512)
        assert len(clean[0][0]) == epc[0] and len(clean[2][0]) == epc[2]
    finally:
        idx.close()
