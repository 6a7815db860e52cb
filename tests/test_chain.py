"""chain_dp parity. CPU: the C restatement (oracle/chain_oracle.c) against the reference scalar kernel's
golden outputs (tests/golden/chain_golden.npz) and, when built, the reference itself. GPU: the HIP
kernel (csrc/chain.hip) against both, bit-exact on scores, parents, targets and peak scores."""
import os

import numpy as np
import pytest

import oracle_lib
from conftest import GOLDEN
from genomicsbench_palisade_amd import gen


@pytest.fixture(scope="module")
def golden():
    z = np.load(os.path.join(GOLDEN, "chain_golden.npz"))
    calls = gen.ChainCalls(z["offsets"], z["x"], z["y"], z["avg_qspan"], z["params4"])
    return calls, [z["scores"], z["parents"], z["targets"], z["peaks"]]


NAMES = ["scores", "parents", "targets", "peak_scores"]


def assert_same(got, exp):
    for k, name in enumerate(NAMES):
        bad = np.nonzero(got[k] != exp[k])[0]
        assert len(bad) == 0, f"{name}: {len(bad)} mismatches, first at {bad[:5]}: {got[k][bad[:5]]} vs {exp[k][bad[:5]]}"


def test_oracle_vs_golden(golden):
    calls, exp = golden
    got = oracle_lib.chain_oracle(calls)
    assert_same(got, exp)
    assert got[4] > calls.nanchors  # visited pairs


def test_oracle_vs_reference_live():
    lib = oracle_lib.ref_chain()
    if lib is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    calls = gen.chain_dataset("small", num_calls=120, seed=77, median_n=800, max_n=30000)
    assert_same(oracle_lib.chain_oracle(calls), oracle_lib.ref_chain_run(lib, calls))


@pytest.mark.gpu
def test_gpu_vs_golden(golden):
    from genomicsbench_palisade_amd import chain, set_device
    set_device(0)
    calls, exp = golden
    b = chain.ChainBatch(calls)
    b.run()
    got = b.results()
    assert_same(got, exp)
    assert got[4] == oracle_lib.chain_oracle(calls)[4]
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("rows", ["1", "0"])
@pytest.mark.parametrize("seed,ncalls,median,maxn", [(1, 300, 1500, 87271), (2, 2000, 200, 5000)])
def test_gpu_vs_oracle(seed, ncalls, median, maxn, rows, monkeypatch):
    """rows "1": sorted calls on chain_rows (two calls per wave), "0": chain_kernel for every block."""
    from genomicsbench_palisade_amd import chain, set_device
    set_device(0)
    monkeypatch.setenv("GB_CHAIN_ROWS", rows)
    calls = gen.chain_dataset("small", num_calls=ncalls, seed=seed, median_n=median, max_n=maxn)
    exp = oracle_lib.chain_oracle(calls, 8)
    b = chain.ChainBatch(calls)
    b.run()
    got = b.results()
    assert_same(got, exp)
    assert got[4] == exp[4]
    b.run()
    assert_same(b.results(), exp)  # re-run on the same device buffers
    b.close()


@pytest.mark.gpu
def test_gpu_cli_dropin(golden, tmp_path):
    """bin/chain (CLI of minimap2-acceleration kernel/scalar main.cpp over host_chain_kernel from
    libgb_chain_dropin.so): read_call input -> print_return output equal to the reference's."""
    import subprocess
    from conftest import ROOT
    calls, exp = golden
    fin, fout = tmp_path / "in.txt", tmp_path / "out.txt"
    gen.write_chain_file(fin, calls)
    exe = os.path.join(ROOT, "genomicsbench_palisade_amd", "bin", "chain")
    r = subprocess.run([exe, "-i", str(fin), "-o", str(fout), "-t", "4"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Time in kernel" in r.stderr
    toks = fout.read_text().split("EOR\n")
    assert toks[-1] == "" and len(toks) == calls.ncalls + 1
    sc, par = [], []
    for c, blk in enumerate(toks[:-1]):
        lines = blk.strip("\n").split("\n")
        assert int(lines[0]) == calls.offsets[c + 1] - calls.offsets[c]
        for ln in lines[1:]:
            a, b = ln.split("\t")
            sc.append(int(a))
            par.append(int(b))
    assert (np.array(sc) == exp[0]).all() and (np.array(par) == exp[1]).all()


def _concat_calls(parts):
    offs = [0]
    for p in parts:
        offs.extend((offs[-1] + p.offsets[1:]).tolist())
    return gen.ChainCalls(np.array(offs, np.int64), np.concatenate([p.x for p in parts]),
                          np.concatenate([p.y for p in parts]), np.concatenate([p.avg_qspan for p in parts]),
                          np.concatenate([p.params4 for p in parts]))


def _cloud_call(rng, n, diagonals, spread, step, noise, span=15):
    """Dense anchors on a few parallel noisy diagonals (competing chains in every window)."""
    x = (np.cumsum(rng.integers(step[0], step[1] + 1, n)) + 1000).astype(np.uint64)
    offs = rng.integers(-spread, spread, diagonals)
    y = np.maximum(x.astype(np.int64) + offs[rng.integers(0, diagonals, n)] + rng.integers(-noise, noise + 1, n), 0)
    yy = (np.uint64(span) << np.uint64(32)) | y.astype(np.uint64)
    return gen.ChainCalls(np.array([0, n]), x, yy, np.array([15.0], np.float32),
                          np.array([[5000, 5000, 500, 1]], np.int32))


def split_set(seed):
    """Long minimap2-shaped calls, dense multi-diagonal clouds (windows of > 1 000 anchors) and one
    long call with unsorted x (never split), for the speculative-segment path."""
    rng = np.random.default_rng(seed)
    parts = [gen.chain_dataset("small", num_calls=40, seed=seed, median_n=3000, max_n=40000)]
    parts.append(_cloud_call(rng, 12000, 4, 300, (1, 6), 3))
    parts.append(_cloud_call(rng, 9000, 16, 450, (0, 2), 3))
    u = gen.chain_dataset("small", num_calls=1, seed=seed + 1, median_n=20000, max_n=20000)
    k = np.arange(u.nanchors)
    k[100:110] = k[100:110][::-1]  # x no longer sorted
    parts.append(gen.ChainCalls(u.offsets, u.x[k], u.y[k], u.avg_qspan, u.params4))
    return _concat_calls(parts)


@pytest.fixture(scope="module")
def split_calls():
    calls = split_set(21)
    return calls, oracle_lib.chain_oracle(calls, 8)


@pytest.mark.gpu
@pytest.mark.parametrize("split,fault,rows", [("", 0, "1"), ("0", 0, "1"), ("256,0", 0, "1"), ("64,0", 0, "1"),
                                              ("128,8", 37, "1"), ("", 997, "1"), ("", 0, "0"), ("128,8", 37, "0"),
                                              ("256,32,0,16", 0, "1"), ("-1,128,0,5000", 0, "1")])
def test_gpu_split_exact(split_calls, monkeypatch, split, fault, rows):
    """Long calls as speculative segments (csrc/chain_split.hip) give the sequential loop's results
    bit for bit: default and tiny segments, no warm-up, injected wrong guesses that the verification
    must catch and the sequential fix-up repair, a 16-anchor window cap (blocks start far inside
    their first anchor's window, so guesses fail for real) and the uncapped window."""
    from genomicsbench_palisade_amd import chain, set_device
    set_device(0)
    calls, exp = split_calls
    monkeypatch.setenv("GB_CHAIN_SPLIT", split)
    monkeypatch.setenv("GB_CHAIN_SPLIT_FAULT", str(fault))
    monkeypatch.setenv("GB_CHAIN_ROWS", rows)
    # equal segments of `seg` (the per-call row target has test_gpu_split_row_target)
    monkeypatch.setenv("GB_CHAIN_TARGET", "0")
    b = chain.ChainBatch(calls)
    b.run()
    got = b.results()
    assert_same(got, exp)
    assert got[4] == exp[4]
    ns, rounds, fixups = b.split_stats()
    if split == "0":
        assert ns == 0
    else:
        # default: the segment length adapts to the batch (512..4096 anchors, chain_split.hip)
        seg = int(split.split(",")[0]) if split and not split.startswith("-") else 512
        long_calls = sum(1 for c in range(calls.ncalls) if calls.offsets[c + 1] - calls.offsets[c] >= 2 * seg)
        assert 0 < ns < long_calls  # the unsorted long call stays whole
    if fault:
        assert fixups > 0 and rounds > 1
    b.run()  # re-run on the same buffers
    assert_same(b.results(), exp)
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("split,fault", [("", 0), ("128,8", 37)])
def test_gpu_split_wave_verification(split_calls, monkeypatch, split, fault):
    """GB_CHAIN_VLANES=0: every split anchor verified by verify_kernel (64 lanes per candidate block)
    instead of verify_lanes (one lane per anchor, verify_kernel only for loops past 64 candidates)."""
    from genomicsbench_palisade_amd import chain, set_device
    set_device(0)
    calls, exp = split_calls
    monkeypatch.setenv("GB_CHAIN_SPLIT", split)
    monkeypatch.setenv("GB_CHAIN_SPLIT_FAULT", str(fault))
    monkeypatch.setenv("GB_CHAIN_VLANES", "0")
    b = chain.ChainBatch(calls)
    b.run()
    got = b.results()
    assert_same(got, exp)
    assert got[4] == exp[4]
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("split,fault", [("512,64", 53), ("1024,0", 211)])
def test_gpu_split_remark_wide_windows(monkeypatch, split, fault):
    """Calls whose windows hold up to max_iter (5000) anchors and whose parent links reach far back,
    with injected wrong guesses: every split call fails at least once, so its targets marks and
    visited counts come from the re-mark pass, whose stamp ring must hold a whole window (a 1 K ring
    lets an anchor's mark overwrite its own earlier one). Targets and visited are asserted with the
    scores, parents and peaks."""
    from genomicsbench_palisade_amd import chain, set_device
    set_device(0)
    rng = np.random.default_rng(91)
    calls = _concat_calls([_cloud_call(rng, 14000, 24, 2000, (0, 1), 40),
                           _cloud_call(rng, 8000, 3, 100, (0, 3), 2),
                           _cloud_call(rng, 6000, 40, 4000, (0, 1), 200)])
    exp = oracle_lib.chain_oracle(calls, 8)
    monkeypatch.setenv("GB_CHAIN_SPLIT", split)
    monkeypatch.setenv("GB_CHAIN_SPLIT_FAULT", str(fault))
    b = chain.ChainBatch(calls)
    b.run()
    got = b.results()
    assert_same(got, exp)
    assert got[4] == exp[4]
    ns, rounds, fixups = b.split_stats()
    assert ns == calls.ncalls and fixups >= ns and rounds > 1
    b.close()


def _long_window_call(rng, n, frac_chain):
    """x step 1, so every window holds max_iter (5 000) anchors; most anchors have dq <= 0 against
    their predecessors (filtered, no parents, no marks), so loops rarely break and visit far more than
    64 candidates: chain_rows' HBM path (candidates older than its 64-anchor ring, global marks)."""
    x = (np.arange(n) + 1000).astype(np.uint64)
    y = rng.integers(0, 1 << 20, n).astype(np.int64)
    on = rng.random(n) < frac_chain
    y[on] = x[on].astype(np.int64) + rng.integers(-3, 4, int(on.sum()))
    yy = (np.uint64(15) << np.uint64(32)) | y.astype(np.uint64)
    return gen.ChainCalls(np.array([0, n]), x, yy, np.array([15.0], np.float32),
                          np.array([[5000, 5000, 500, 1]], np.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("split", ["0", "1024,64"])
def test_gpu_rows_long_windows(monkeypatch, split):
    """chain_rows past its ring: visited counts far above 64, marks from HBM, whole and split calls."""
    from genomicsbench_palisade_amd import chain, set_device
    set_device(0)
    rng = np.random.default_rng(5)
    calls = _concat_calls([_long_window_call(rng, 9000, 0.05), _long_window_call(rng, 7000, 0.3),
                           _long_window_call(rng, 3000, 0.8), _cloud_call(rng, 6000, 40, 4000, (0, 1), 200)])
    exp = oracle_lib.chain_oracle(calls, 8)
    assert exp[4] > 64 * calls.nanchors // 4  # the HBM path is exercised
    monkeypatch.setenv("GB_CHAIN_SPLIT", split)
    monkeypatch.setenv("GB_CHAIN_ROWS", "1")
    b = chain.ChainBatch(calls)
    b.run()
    got = b.results()
    assert_same(got, exp)
    assert got[4] == exp[4]
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("target,segmin,fault", [("600", "", 0), ("300", "", 0), ("0", "", 0), ("600", "16", 37)])
def test_gpu_split_row_target(target, segmin, fault, monkeypatch):
    """Per-call segment lengths under a row target (GB_CHAIN_TARGET; a batch under 1 M anchors takes
    600 by default, with segments of >= 64 anchors and a 16-anchor warm-up): calls longer than the
    target split into segments as long as their window leaves room for, shorter ones run whole --
    bit-exact against the oracle either way, also with 16-anchor segments and injected wrong guesses."""
    from genomicsbench_palisade_amd import chain, set_device
    set_device(0)
    monkeypatch.setenv("GB_CHAIN_TARGET", target)
    if segmin:
        monkeypatch.setenv("GB_CHAIN_SEGMIN", segmin)
    monkeypatch.setenv("GB_CHAIN_SPLIT_FAULT", str(fault))
    calls = gen.chain_dataset("small", num_calls=300, seed=31, median_n=1500, max_n=30000)
    exp = oracle_lib.chain_oracle(calls, 8)
    b = chain.ChainBatch(calls)
    b.run()
    got = b.results()
    assert_same(got, exp)
    assert got[4] == exp[4]
    if target != "0":
        ns, rounds, fixups = b.split_stats()
        assert ns > 0
        if fault:
            assert fixups > 0 and rounds > 1
    b.close()
