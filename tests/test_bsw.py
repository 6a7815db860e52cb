"""Banded SW parity. CPU: the C restatement (oracle/bsw_oracle.c) against the golden outputs of bwa v1
ksw_extend2 -- the function the benchmark's scalarBandedSWA (bandedSWA.cpp:130-251) restates --
(tests/golden/bsw_golden.npz, six parameter sets) and, when built, against ksw_extend2 live. GPU: the
HIP kernel (csrc/bsw.hip) bit-exact on score/qle/tle/gtle/gscore/max_off and on the DP cell count."""
import ctypes
import os

import numpy as np
import pytest

import oracle_lib
from conftest import GOLDEN
from genomicsbench_palisade_amd import bsw, gen

FIELDS = bsw.OUT_FIELDS


@pytest.fixture(scope="module")
def golden():
    z = np.load(os.path.join(GOLDEN, "bsw_golden.npz"))
    p = gen.BswPairs(z["tgt"], z["toff"], z["tlen"], z["qry"], z["qoff"], z["qlen"], z["h0"])
    sets = {}
    for k in z.files:
        if k.endswith("_out"):
            name = k[:-4]
            par = z[name + "_params"]
            mat = z[name + "_mat"]
            P = bsw.Params(*[int(v) for v in par])
            for i in range(25):
                P.mat[i] = int(mat[i])
            sets[name] = (P, z[k])
    return p, sets


def assert_same(got, exp, what=""):
    bad = np.nonzero((got != exp).any(axis=1))[0]
    if len(bad):
        b = bad[0]
        raise AssertionError(f"{what}: {len(bad)} pairs differ; first pair {b}: got "
                             f"{dict(zip(FIELDS, got[b].tolist()))} expected {dict(zip(FIELDS, exp[b].tolist()))}")


def test_params_match_benchmark_defaults():
    p = bsw.default_params()
    assert (p.o_del, p.e_del, p.o_ins, p.e_ins, p.zdrop, p.end_bonus, p.w) == (6, 1, 6, 1, 100, 5, 100)
    m = p.mat_array().reshape(5, 5)
    assert (np.diag(m)[:4] == 1).all() and m[0, 1] == -4 and (m[4] == -1).all() and (m[:, 4] == -1).all()


def test_oracle_vs_golden(golden):
    p, sets = golden
    assert len(sets) == 6
    for name, (P, exp) in sets.items():
        got, cells, tot = oracle_lib.bsw_oracle(p, P)
        assert_same(got, exp, name)
        assert tot == cells.sum() > 0


def test_oracle_vs_reference_live():
    lib = oracle_lib.ref_bsw()
    if lib is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    p = gen.bsw_pairs(20000, seed=123)
    for kw in ({}, {"w": 3}, {"zdrop": 1}):
        P = bsw.default_params(**kw)
        assert_same(oracle_lib.bsw_oracle(p, P)[0], oracle_lib.ref_bsw_run(lib, p, P), str(kw))


def test_pair_file_roundtrip(tmp_path):
    """write_bsw_file emits the loadPairs format (main_banded.cpp:160-202): h0, ref, query lines."""
    p = gen.bsw_pairs(50, seed=5)
    f = tmp_path / "pairs.txt"
    gen.write_bsw_file(f, p)
    lines = f.read_bytes().split(b"\n")
    assert len(lines) == 3 * p.n + 1 and lines[-1] == b""
    for k in range(p.n):
        assert int(lines[3 * k]) == p.h0[k]
        t = np.frombuffer(lines[3 * k + 1], np.uint8) - 48
        q = np.frombuffer(lines[3 * k + 2], np.uint8) - 48
        assert (t == p.tgt[p.toff[k]:p.toff[k] + p.tlen[k]]).all()
        assert (q == p.qry[p.qoff[k]:p.qoff[k] + p.qlen[k]]).all()


def test_seqpair_layout():
    assert bsw.SEQPAIR_DTYPE.itemsize == 72
    assert ctypes.sizeof(bsw.Params) == 7 * 4 + 25 + 3


# ---------------------------------------------------------------- GPU

def _gpu(p, P):
    from genomicsbench_palisade_amd import set_device
    set_device(0)
    b = bsw.BswBatch(p, P)
    b.run()
    out, cells, tot = b.results()
    b.close()
    return out, cells, tot


@pytest.mark.gpu
@pytest.mark.parametrize("tail", ["0", None])
def test_gpu_vs_golden(golden, monkeypatch, tail):
    """tail "0": every pair on the pair-per-lane kernels; None: the default routing (a batch this
    small runs on the wave-per-pair kernel)."""
    if tail is not None:
        monkeypatch.setenv("GB_BSW_TAIL", tail)
    p, sets = golden
    for name, (P, exp) in sets.items():
        got, cells, tot = _gpu(p, P)
        assert_same(got, exp, name)
        ocells = oracle_lib.bsw_oracle(p, P)[1]
        assert (cells == ocells).all(), f"{name}: cell counts differ on {(cells != ocells).sum()} pairs"
        assert tot == ocells.sum()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,qlen,extra", [(1, 100000, (10, 150), (0, 100)), (2, 20000, (150, 255), (0, 400)),
                                               (3, 20000, (1, 70), (0, 1500))])
@pytest.mark.parametrize("tail", ["0", None])
def test_gpu_vs_oracle(seed, n, qlen, extra, tail, monkeypatch):
    if tail is not None:
        monkeypatch.setenv("GB_BSW_TAIL", tail)
    p = gen.bsw_pairs(n, seed=seed, qlen=qlen, extra=extra)
    P = bsw.default_params()
    got, cells, tot = _gpu(p, P)
    exp, ocells, otot = oracle_lib.bsw_oracle(p, P, nthreads=8)
    assert_same(got, exp, f"seed {seed}")
    assert (cells == ocells).all() and tot == otot


@pytest.mark.gpu
@pytest.mark.parametrize("h0step,qshift", [("0", "2"), ("3", "0"), ("8", "6"), ("40", "3")])
def test_gpu_grouping_key_does_not_change_results(monkeypatch, h0step, qshift):
    """The batch's sort key (variant, h0 == 0, query length step, h0 step, target length) only orders
    pairs into waves; every grouping must give the oracle's outputs and cell counts, scattered back to
    the caller's order (pairs with h0 0, large h0 and every variant in the set)."""
    monkeypatch.setenv("GB_BSW_H0STEP", h0step)
    monkeypatch.setenv("GB_BSW_QSHIFT", qshift)
    monkeypatch.setenv("GB_BSW_TAIL", "0.1")  # the lane kernels (a batch this small would go to the wave kernel)
    p = gen.bsw_pairs(30000, seed=17, qlen=(1, 160), extra=(0, 200))
    p.h0[::7] = 0
    p.h0[1::11] = 200
    P = bsw.default_params()
    got, cells, tot = _gpu(p, P)
    exp, ocells, otot = oracle_lib.bsw_oracle(p, P, nthreads=8)
    assert_same(got, exp, f"h0 step {h0step}, query shift {qshift}")
    assert (cells == ocells).all() and tot == otot


@pytest.mark.gpu
def test_gpu_get_scores16_and_repeat():
    from genomicsbench_palisade_amd import set_device
    set_device(0)
    p = gen.bsw_pairs(5000, seed=9)
    P = bsw.default_params()
    sp = bsw.get_scores16(p, P)
    exp = oracle_lib.bsw_oracle(p, P)[0]
    got = np.stack([sp[f] for f in FIELDS], axis=1)
    assert_same(got, exp, "get_scores16")
    assert (sp["id"] == np.arange(p.n)).all() and (sp["seqid"] == -1).all()
    b = bsw.BswBatch(p, P)
    outs = []
    for _ in range(3):
        b.run()
        outs.append(b.results()[0])
    assert all((o == outs[0]).all() for o in outs)
    assert b.timing() > 0
    b.close()


@pytest.mark.gpu
def test_gpu_rejects_bad_pairs():
    from genomicsbench_palisade_amd import GbError, set_device
    set_device(0)
    P = bsw.default_params()
    for ql in (0, 256):
        q = np.zeros(max(ql, 1), np.uint8)
        p = gen.BswPairs(np.zeros(4, np.uint8), np.zeros(1, np.int64), np.array([4], np.int32), q,
                         np.zeros(1, np.int64), np.array([ql], np.int32), np.array([10], np.int32))
        with pytest.raises(GbError):
            bsw.BswBatch(p, P)
    p = gen.BswPairs(np.zeros(4, np.uint8), np.array([2], np.int64), np.array([4], np.int32), np.zeros(4, np.uint8),
                     np.zeros(1, np.int64), np.array([4], np.int32), np.array([10], np.int32))
    with pytest.raises(GbError):
        bsw.BswBatch(p, P)
    empty = gen.BswPairs(np.zeros(0, np.uint8), np.zeros(0, np.int64), np.zeros(0, np.int32), np.zeros(0, np.uint8),
                         np.zeros(0, np.int64), np.zeros(0, np.int32), np.zeros(0, np.int32))
    out, cells, tot = _gpu(empty, P)
    assert out.shape == (0, 6) and tot == 0


@pytest.mark.gpu
def test_gpu_cli_dropin(golden, tmp_path):
    """bin/bsw (CLI of main_banded.cpp over BandedPairWiseSW::getScores16 from libgb_bsw_dropin.so)
    on a loadPairs-format file reproduces ksw_extend2's outputs."""
    import subprocess
    from conftest import ROOT
    p, sets = golden
    P, exp = sets["default"]
    fin, fout = tmp_path / "pairs.txt", tmp_path / "out.tsv"
    gen.write_bsw_file(fin, p)
    exe = os.path.join(ROOT, "genomicsbench_palisade_amd", "bin", "bsw")
    r = subprocess.run([exe, "-pairs", str(fin), "-t", "1", "-b", "512", "-o", str(fout)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    assert f"Total Pairs processed: {p.n}" in r.stdout
    got = np.loadtxt(fout, dtype=np.int32, ndmin=2)
    assert_same(got, exp, "bsw CLI")


def reference_outputs(p, P):
    """ksw_extend2 from the reference tree when built (oracle/_ref), else the restatement."""
    lib = oracle_lib.ref_bsw()
    return oracle_lib.ref_bsw_run(lib, p, P) if lib is not None else oracle_lib.bsw_oracle(p, P)[0]


def outs_of(sp):
    return np.stack([sp[f] for f in FIELDS], axis=1)


def eight_bit_pairs(n, seed):
    """Pairs inside the 8-bit kernel's domain (bwamem.cpp:2152-2155): len1, len2 < 128 and
    h0 + min(len1, len2) < 128 (match score 1), including the boundary values."""
    p = gen.bsw_pairs(n, seed=seed, qlen=(1, 120), extra=(0, 7))
    h0 = p.h0.copy()
    lim = 127 - np.minimum(p.tlen, p.qlen)
    h0 = np.minimum(h0, lim).astype(np.int32)
    h0[::7] = lim[::7]  # h0 + min(len1, len2) == 127
    return gen.BswPairs(p.tgt, p.toff, p.tlen, p.qry, p.qoff, p.qlen, h0)


@pytest.mark.gpu
def test_gpu_scores8_domain_exact_and_refusal():
    """getScores8 (bandedSWA.cpp:426-725): pairs of the 8-bit domain are bit-exact against the reference
    ksw_extend2 (and the 16-bit path); a call holding one pair outside the domain is refused and writes
    nothing."""
    from genomicsbench_palisade_amd import GbError, set_device
    set_device(0)
    p = eight_bit_pairs(6000, 71)
    assert p.tlen.max() < 128 and p.qlen.max() < 128
    params = bsw.default_params()
    exp = reference_outputs(p, params)
    sp = bsw.get_scores8(p, params)
    assert_same(outs_of(sp), exp, "getScores8")
    for bad in ("len1", "len2", "h0"):
        q = p.subset(np.arange(50))
        if bad == "len1":
            q = gen.concat_bsw([q, gen.bsw_pairs(1, seed=3, qlen=(20, 20), extra=(110, 110))])
        elif bad == "len2":
            q = gen.concat_bsw([q, gen.bsw_pairs(1, seed=3, qlen=(128, 128), extra=(0, 0))])
        else:
            q.h0 = q.h0.copy()
            q.h0[10] = 128 - min(int(q.tlen[10]), int(q.qlen[10]))
        with pytest.raises(GbError, match="8-bit"):
            bsw.get_scores8(q, params)


@pytest.mark.gpu
def test_gpu_cli_scores8(tmp_path):
    """bin/bsw -bits 8 runs BandedPairWiseSW::getScores8 of the drop-in on a loadPairs file."""
    import subprocess
    from conftest import ROOT
    p = eight_bit_pairs(3000, 72)
    exp = reference_outputs(p, bsw.default_params())
    fin, fout = tmp_path / "pairs.txt", tmp_path / "out.tsv"
    gen.write_bsw_file(fin, p)
    exe = os.path.join(ROOT, "genomicsbench_palisade_amd", "bin", "bsw")
    r = subprocess.run([exe, "-pairs", str(fin), "-t", "1", "-b", "512", "-bits", "8", "-o", str(fout)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    assert_same(np.loadtxt(fout, dtype=np.int32, ndmin=2), exp, "bsw CLI -bits 8")
    bad = gen.bsw_pairs(20, seed=5, qlen=(130, 140))
    gen.write_bsw_file(fin, bad)
    r = subprocess.run([exe, "-pairs", str(fin), "-bits", "8"], capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "8-bit" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("limit", ["0", "100000000"])
def test_gpu_get_scores16_small_and_batch_paths(golden, monkeypatch, limit):
    """getScores16's two paths -- the pair-per-lane batch launch (GB_BSW_SMALL=0) and the small-call
    path (packed pinned staging + the wave-per-pair kernel for every pair, used below GB_BSW_SMALL
    pairs) -- both reproduce ksw_extend2 on the golden sets (six parameter sets) and on long queries
    and targets."""
    from genomicsbench_palisade_amd import GbError, set_device
    set_device(0)
    monkeypatch.setenv("GB_BSW_SMALL", limit)
    p, sets = golden
    for name, (P, exp) in sets.items():
        sp = bsw.get_scores16(p, P)
        assert_same(np.stack([sp[f] for f in FIELDS], axis=1), exp, f"{name} (limit {limit})")
    q = gen.bsw_pairs(3000, seed=17, qlen=(120, 255), extra=(0, 900))
    P = bsw.default_params()
    sp = bsw.get_scores16(q, P)
    assert_same(np.stack([sp[f] for f in FIELDS], axis=1), oracle_lib.bsw_oracle(q, P, nthreads=8)[0], "long")
    bad = gen.BswPairs(np.zeros(4, np.uint8), np.array([2], np.int64), np.array([4], np.int32), np.zeros(4, np.uint8),
                       np.zeros(1, np.int64), np.array([4], np.int32), np.array([10], np.int32))
    with pytest.raises(GbError):
        bsw.get_scores16(bad, P)


@pytest.mark.gpu
def test_gpu_dropin_512_pair_batches_from_threads():
    """BandedPairWiseSW::getScores16 called per 512-pair batch from 8 host threads (one object each), each
    batch's idr/idq indexing its own buffers, as main_banded.cpp:896-924 calls it
    (tests/cpp/dropin_bench.cpp): every pair equals ksw_extend2."""
    import ctypes
    from conftest import ROOT
    from genomicsbench_palisade_amd import set_device
    set_device(0)
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "_build", "libdropin_bench.so"))
    vp = ctypes.c_void_p
    lib.bench_bsw_batches.argtypes = [vp, vp, ctypes.c_int64, vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]
    lib.bench_bsw_batches.restype = ctypes.c_double
    p = gen.bsw_pairs(20000, seed=23)
    P = bsw.default_params()
    sp = bsw.seqpairs(p)
    par7, mat = P.as_array(), P.mat_array()
    got = np.zeros((p.n, 6), np.int32)
    t = lib.bench_bsw_batches(par7.ctypes.data, mat.ctypes.data, p.n, sp.ctypes.data, p.tgt.ctypes.data,
                              p.qry.ctypes.data, 512, 8, got.ctypes.data)
    assert t > 0
    assert_same(got, oracle_lib.bsw_oracle(p, P, nthreads=8)[0], "512-pair batches")
