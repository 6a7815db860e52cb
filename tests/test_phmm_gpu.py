"""GPU parity: the HIP PairHMM path (libgb.so, csrc/phmm.hip) against the reference golden vectors
and the oracle -- bit-exact raw f32/f64 probabilities and final log10 likelihoods (host log10);
the device log10 epilogue within 1 ulp (north_star tolerance for PairHMM log-likelihoods)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, assert_phmm_exact, bits
from genomicsbench_palisade_amd import gen
from genomicsbench_palisade_amd._tc import TestcaseArray

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def phmm():
    from genomicsbench_palisade_amd import phmm, set_device
    set_device(0)
    phmm.init_pairhmm()
    return phmm


def oracle_run(ta):
    import oracle_lib
    o = oracle_lib.oracle()
    n = ta.n
    out, rf, rd = np.zeros(n), np.zeros(n, np.float32), np.zeros(n)
    ud = np.zeros(n, np.int32)
    o.phmm_oracle_batch(ctypes.addressof(ta.arr), n, out.ctypes.data, rf.ctypes.data, rd.ctypes.data,
                        ud.ctypes.data, 16)
    return out, rf, rd, ud


def assert_exact(got, expect):
    """Everything computelikelihoodsboth exposes, bit for bit (conftest.assert_phmm_exact)."""
    return assert_phmm_exact(got, expect)


def assert_raw_exact(got, expect):
    """Raw f32 of every testcase too: the f32 pass without its early exit (GB_PHMM_EXIT=0)."""
    for k, name in enumerate(("log10", "raw f32", "raw f64")):
        bad = np.nonzero(bits(got[k]) != bits(expect[k]))[0]
        assert len(bad) == 0, f"{name} mismatch at {bad[:10]}: {got[k][bad[:5]]} vs {expect[k][bad[:5]]}"


@pytest.mark.parametrize("which", ["cross", "pairs"])
def test_golden_bit_exact(phmm, phmm_golden, which):
    got = phmm.compute_likelihoods_both(phmm_golden[which])
    assert_exact(got, phmm_golden[which + "_expect"])


def test_kat(phmm):
    ta = TestcaseArray.from_pairs([((b"ACGT", b"++++", b"++++", b"++++", b"++++"), b"ACGT")])
    res = phmm.compute_likelihoods_both(ta)[0]
    assert res[0] == -0.6022796630859375


def test_golden_raw_f32_without_exit(phmm, phmm_golden, monkeypatch):
    """With the early exit off every raw f32 value is the reference's, also below MIN_ACCEPTED."""
    monkeypatch.setenv("GB_PHMM_EXIT", "0")
    for which in ("cross", "pairs"):
        assert_raw_exact(phmm.compute_likelihoods_both(phmm_golden[which]), phmm_golden[which + "_expect"])


def test_compute_f32_full(phmm):
    """computelikelihoodsfloat's path (gb_phmm_compute_f32): the full raw f32 of every testcase, the
    ones that fall back included, on a job where the early exit drops some."""
    rng = np.random.default_rng(41)
    ta = TestcaseArray.from_batches([gen.phmm_batch(rng, 40, 16) for _ in range(3)])
    exp = oracle_run(ta)
    assert (exp[1] < 1e-28).sum() > 0
    assert (bits(phmm.compute_f32(ta)) == bits(exp[1])).all()


def test_early_exit_drops_and_stays_exact(phmm, monkeypatch):
    """The early exit (phmm_stack kExit) drops testcases on a job shaped like the bench's (reads that
    fall back by far), the outputs computelikelihoodsboth exposes stay bit-exact, and with the exit
    off the same job reproduces every raw f32 value."""
    rng = np.random.default_rng(43)
    ta = TestcaseArray.from_batches([gen.phmm_batch(rng, 64, 32) for _ in range(4)])
    exp = oracle_run(ta)
    bad = assert_exact(phmm.compute_likelihoods_both(ta), exp)
    assert bad["f32_dropped"] > 0, bad
    monkeypatch.setenv("GB_PHMM_EXIT", "0")
    assert_raw_exact(phmm.compute_likelihoods_both(ta), exp)


@pytest.mark.parametrize("seed,kind", [(1, "large"), (2, "small"), (3, "long")])
def test_random_vs_oracle(phmm, seed, kind):
    rng = np.random.default_rng(seed)
    if kind == "large":
        b = gen.phmm_batch(rng, 64, 32)
    elif kind == "small":
        b = gen.phmm_batch(rng, 40, 20, hap_max=302)
    else:  # long haplotypes / reads beyond the benchmark shapes
        b = gen.phmm_batch(rng, 6, 5, read_len=(300, 700), hap_max=2000)
    ta = TestcaseArray.from_batch(b)
    assert_exact(phmm.compute_likelihoods_both(ta), oracle_run(ta))


def test_device_epilogue_within_1ulp(phmm):
    rng = np.random.default_rng(7)
    ta = TestcaseArray.from_batch(gen.phmm_batch(rng, 50, 20))
    db = phmm.DeviceBatch(ta)
    db.run()
    res, rf, rd, ud, dev = db.results()
    # north_star: "within 1 ulp float". The device log10f/log10 may differ from glibc by 1 ulp of the
    # log10 value L itself; result = round(L - LOG10_INITIAL_CONSTANT), so the bound is
    # ulp(L) + ulp(result) in the precision of the path that produced the result.
    u = ud.astype(bool)
    f32 = lambda x: np.spacing(np.abs(np.asarray(x, np.float32))).astype(np.float64)
    with np.errstate(divide="ignore"):
        Lf = np.log10(rf.astype(np.float64))
        Ld = np.log10(np.where(u, rd, 1.0))
    tol = np.where(u, np.spacing(np.abs(Ld)) + np.spacing(np.abs(res)), f32(Lf) + f32(res))
    bad = np.nonzero(~(np.abs(dev - res) <= tol))[0]
    assert len(bad) == 0, [(int(k), float(res[k]), float(dev[k]), float(rf[k]), float(rd[k]), int(ud[k]))
                           for k in bad[:8]]
    assert (dev == res).mean() > 0.5
    t, cells, nf64 = db.stats()
    assert t == ta.n and nf64 == int(ud.sum())
    db.close()


def test_repeat_runs_identical(phmm):
    rng = np.random.default_rng(11)
    ta = TestcaseArray.from_batch(gen.phmm_batch(rng, 30, 30))
    db = phmm.DeviceBatch(ta)
    db.run()
    a = db.results()
    db.run()
    db.run()
    b = db.results()
    for x, y in zip(a, b):
        assert (x == y).all()
    db.close()


def test_compute_f64_all(phmm, phmm_golden):
    import oracle_lib
    ta = phmm_golden["pairs"]
    rd = phmm.compute_f64(ta)
    o = oracle_lib.oracle()
    exp = np.array([o.phmm_oracle_prob_f64(ctypes.addressof(ta.arr[k])) for k in range(ta.n)])
    assert (bits(rd) == bits(exp)).all()


def test_dropin_symbols(phmm_golden):
    """libgkl_pairhmm_c.so exports the reference's C++ entry points; call them via their mangled
    names exactly as a binary linked against GKL would."""
    so = ctypes.CDLL(os.path.join(ROOT, "genomicsbench_palisade_amd", "lib", "libgkl_pairhmm_c.so"))
    so._Z11initPairHMMv()
    so._Z22computelikelihoodsbothP8testcasePdi.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    ta = phmm_golden["cross"]
    out = np.zeros(ta.n)
    so._Z22computelikelihoodsbothP8testcasePdi(ctypes.addressof(ta.arr), out.ctypes.data, ta.n)
    assert (bits(out) == bits(phmm_golden["cross_expect"][0])).all()


def test_phmm_cli(tmp_path):
    """bin/phmm parses the reference's .in format and prints PRINT_OUTPUT lines."""
    rng = np.random.default_rng(5)
    batches = [gen.phmm_batch(rng, 5, 3), gen.phmm_batch(rng, 7, 4, hap_max=302)]
    path = tmp_path / "t.in"
    gen.write_phmm_file(str(path), batches)
    exe = os.path.join(ROOT, "genomicsbench_palisade_amd", "bin", "phmm")
    out = subprocess.run([exe, "-f", str(path), "-p"], capture_output=True, text=True, timeout=300,
                         check=True).stdout
    vals = [float(x) for x in out.split("Num GPUs")[1].splitlines()[1:] if x.strip() and "PairHMM" not in x]
    expect = []
    for b in batches:
        ta = TestcaseArray.from_batch(b)
        expect.extend(oracle_run(ta)[0])
    assert len(vals) == len(expect)
    assert np.allclose(vals, expect, atol=1e-6, rtol=0)  # "%lf" prints 6 decimals
    assert "PairHMM completed. Kernel runtime:" in out


ACGTN = np.frombuffer(b"ACGTN", np.uint8)


def _read(rng, rl):
    b = ACGTN[rng.integers(0, 5, rl)].tobytes()
    q = rng.integers(6, 41, rl).astype(np.uint8).tobytes()
    i = rng.integers(40, 46, rl).astype(np.uint8).tobytes()
    d = rng.integers(40, 46, rl).astype(np.uint8).tobytes()
    c = np.full(rl, 10, np.uint8).tobytes()
    return (b, q, i, d, c)


@pytest.mark.parametrize("seed", [5, 6])
def test_stack_edges_vs_oracle(phmm, seed):
    """Stacked testcases (csrc/phmm.hip phmm_stack): reads of 1, 2, 62-66, 127-129 rows and one taller
    than a stack (> 1024 rows), haplotypes of 1, 3, 63, 64 and 700 columns, many reads per haplotype
    (stacks of up to 64 testcases whose rows start anywhere in a stripe): bit-exact against the
    oracle, f32 and f64 results and the fallback choice."""
    rng = np.random.default_rng(seed)
    lens = [1, 2, 62, 63, 64, 65, 66, 127, 128, 129, 1100] + list(rng.integers(1, 200, 80))
    reads = [_read(rng, int(n)) for n in lens]
    haps = [gen.BASES[rng.integers(0, 4, n)].tobytes() for n in (1, 3, 63, 64, 700, 250)]
    ta = TestcaseArray(reads, haps)  # the cross product: 91 reads per haplotype
    got = phmm.compute_likelihoods_both(ta)
    exp = oracle_run(ta)
    assert_exact(got, exp)


@pytest.mark.parametrize("chunks", ["3", "1", "6"])
def test_pipelined_compute_bit_exact(phmm, monkeypatch, chunks):
    """gb_phmm_compute's pipelined path (chunks of growing size, each on its own workspace and stream,
    the first packed on the calling thread and the rest concurrently on worker threads; GB_PHMM_PIPE
    forces it for a small call, 6 chunks use workspaces beyond the four gb_phmm_init reserves) gives
    the one-job results, against the oracle."""
    monkeypatch.setenv("GB_PHMM_PIPE", chunks)
    rng = np.random.default_rng(23)
    ta = TestcaseArray.from_batches([gen.phmm_batch(rng, 30, 12) for _ in range(5)])
    got = phmm.compute_likelihoods_both(ta)
    assert_exact(got, oracle_run(ta))


def big_pool_job(seed=31, n=600):
    """Every testcase its own long read: ~1.1 KB of packed pool per testcase, far above the 32 B per
    testcase a fill reserves pinned staging for before its pack."""
    rng = np.random.default_rng(seed)
    haps = [gen.BASES[rng.integers(0, 4, k)].tobytes() for k in (300, 410, 77)]
    return TestcaseArray.from_pairs([(_read(rng, int(m)), haps[k % 3])
                                     for k, m in enumerate(rng.integers(150, 260, n))])


def test_pipelined_fresh_workspaces_bit_exact(tmp_path):
    """The first call of a process that reserved nothing at init (GB_PHMM_PREALLOC=0): every chunk's
    fill allocates its device buffers and pinned staging while other chunks' fills and kernels run,
    and the staging grows after the pack (keeping the descriptors already written) -- bit-exact
    against the oracle, in a process of its own."""
    out = tmp_path / "res.npz"
    code = (
        "import sys, numpy as np\n"
        f"sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tests')!r})\n"
        "from genomicsbench_palisade_amd import phmm, set_device\n"
        "import test_phmm_gpu as t\n"
        "set_device(0); phmm.init_pairhmm()\n"
        "r = phmm.compute_likelihoods_both(t.big_pool_job())\n"
        f"np.savez({str(out)!r}, out=r[0], rf=r[1], rd=r[2], ud=r[3])\n")
    env = dict(os.environ, GB_PHMM_PREALLOC="0", GB_PHMM_PIPE="3")
    subprocess.run([os.sys.executable, "-c", code], env=env, check=True, timeout=240)
    z = np.load(out)
    ta = big_pool_job()
    exp = oracle_run(ta)
    assert_exact((z["out"], z["rf"], z["rd"], z["ud"]), exp)


def test_pipelined_big_pool_bit_exact(phmm, monkeypatch):
    """The same shape in this process (workspaces reserved at init), other reads."""
    monkeypatch.setenv("GB_PHMM_PIPE", "3")
    ta = big_pool_job(seed=37)
    assert_exact(phmm.compute_likelihoods_both(ta), oracle_run(ta))


def test_rows_per_lane_ab_identical(phmm, monkeypatch):
    """The f32 pass with one row per lane (default) and with two (GB_PHMM_RPL=2) agree bit for bit
    on a job with many stacks, partial stripes and both passes."""
    rng = np.random.default_rng(29)
    ta = TestcaseArray.from_batches([gen.phmm_batch(rng, 50, 20) for _ in range(4)])
    monkeypatch.setenv("GB_PHMM_EXIT", "0")  # the two-row kernel has no early exit: compare every raw f32
    outs = []
    for rpl in ("1", "2"):
        monkeypatch.setenv("GB_PHMM_RPL", rpl)
        outs.append(phmm.compute_likelihoods_both(ta))
    for a, b in zip(outs[0][:3], outs[1][:3]):
        assert (bits(a) == bits(b)).all()


@pytest.mark.parametrize("where", ["chunk2", "last"])
def test_pipelined_bad_testcase_reports_its_index(phmm, monkeypatch, where):
    """A bad testcase in a later chunk of a pipelined call fails the whole call before any device
    work, and the error names its index in the caller's array (the call is validated on the calling
    thread before it is cut into chunks); the next call on the same workspaces is exact."""
    from genomicsbench_palisade_amd import GbError
    monkeypatch.setenv("GB_PHMM_PIPE", "4")
    rng = np.random.default_rng(47)
    ta = TestcaseArray.from_batches([gen.phmm_batch(rng, 30, 12) for _ in range(4)])
    n = ta.n
    bad = (n * 3 // 10 + 7) if where == "chunk2" else n - 2  # chunk weights 1:2:3:4 of n
    ta.arr[bad].haplen = 70000
    with pytest.raises(GbError, match=f"testcase {bad}: haplen 70000"):
        phmm.compute_likelihoods_both(ta)
    ok = TestcaseArray.from_batches([gen.phmm_batch(rng, 30, 12) for _ in range(4)])
    assert_exact(phmm.compute_likelihoods_both(ok), oracle_run(ok))


@pytest.mark.parametrize("tail", ["0", "0.9:64", "1.0:1", "0.5:300"])
def test_tail_split_stacks_exact(phmm, monkeypatch, tail):
    """The LPT tail split (csrc/phmm.hip batch_fill: the stacks holding the last part of the cost cut
    into shorter stacks; default 10 % into <= 512 rows on jobs of taller stacks) forced over most of a
    job, down to one testcase per stack, with 1024-row stacks before it: bit-exact, both passes."""
    monkeypatch.setenv("GB_PHMM_TAIL", tail)
    monkeypatch.setenv("GB_PHMM_STACK_ROWS", "1024")
    rng = np.random.default_rng(53)
    ta = TestcaseArray.from_batches([gen.phmm_batch(rng, 60, 24) for _ in range(3)])
    exp = oracle_run(ta)
    assert (exp[1] < 1e-28).any()
    assert_exact(phmm.compute_likelihoods_both(ta), exp)
    db = phmm.DeviceBatch(ta)
    db.run()
    assert_exact(db.results()[:4], exp)
    db.close()


@pytest.mark.parametrize("knobs", ["GB_PHMM_F64_PLAN=0", "GB_PHMM_F64_PARTS=2", "GB_PHMM_F64_PARTS=8",
                                   "GB_PHMM_F64_PARTS=3,GB_PHMM_STACK_ROWS=512", "GB_PHMM_F64_PLAN=0,GB_PHMM_F64_PARTS=2"])
def test_f64_plan_exact(phmm, monkeypatch, knobs):
    """The f64 pass's units ordered by cost (csrc/phmm.hip f64_plan / f64_plan_order: only units with
    fallback rows, costliest first; default one unit per stack) against stack order and several
    units per stack -- bit-exact, the fallback count equal, repeated runs of one batch identical."""
    for kv in knobs.split(","):
        k, v = kv.split("=")
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(59)
    ta = TestcaseArray.from_batches([gen.phmm_batch(rng, 50, 20) for _ in range(4)])
    exp = oracle_run(ta)
    nfb = int((exp[1] < 1e-28).sum())
    assert nfb > 0
    db = phmm.DeviceBatch(ta)
    try:
        for _ in range(2):
            db.run()
            assert_exact(db.results()[:4], exp)
            assert db.stats()[2] == nfb
    finally:
        db.close()
