"""Chain backtrack parity (minimap2's consumer of chain_dp's score / parent / peak).
CPU: the C restatement (oracle/chain_oracle.c chain_oracle_backtrack, after the DP restatement)
against the reference testbed mm_chain_dp's chains in tests/golden/chain_bt_golden.npz and, when
built here, the reference itself (oracle/_ref/libref_chain_bt.so). GPU: csrc/chain_bt.hip on the
HIP chain_dp outputs against both, bit-exact on the chains (score << 32 | count, output order) and
their anchors."""
import os

import numpy as np
import pytest

import oracle_lib
from conftest import GOLDEN
from genomicsbench_palisade_amd import gen


@pytest.fixture(scope="module")
def golden():
    z = np.load(os.path.join(GOLDEN, "chain_bt_golden.npz"))
    calls = gen.ChainCalls(z["offsets"], z["x"], z["y"], z["avg_qspan"], z["params4"])
    exp = []
    for k, (mc, ms) in enumerate(z["bt_params"]):
        nch, nan = z[f"nch{k}"], z[f"nan{k}"]
        cu, ca = np.concatenate([[0], np.cumsum(nch)]), np.concatenate([[0], np.cumsum(nan)])
        us = [z[f"u{k}"][cu[c]:cu[c + 1]] for c in range(calls.ncalls)]
        an = [(z[f"bx{k}"][ca[c]:ca[c + 1]], z[f"by{k}"][ca[c]:ca[c + 1]]) for c in range(calls.ncalls)]
        exp.append((int(mc), int(ms), us, an))
    return calls, exp


def same_chains(calls, got_us, got_an, exp_us, exp_an):
    bad = [c for c in range(calls.ncalls)
           if not (np.array_equal(got_us[c], exp_us[c]) and np.array_equal(got_an[c][0], exp_an[c][0])
                   and np.array_equal(got_an[c][1], exp_an[c][1]))]
    assert not bad, f"{len(bad)} calls differ, first {bad[:5]}: {got_us[bad[0]][:4]} vs {exp_us[bad[0]][:4]}"


def test_oracle_vs_golden(golden):
    calls, exp = golden
    f, p, _, v, _ = oracle_lib.chain_oracle(calls)
    for mc, ms, us, an in exp:
        _, gus, gan = oracle_lib.chain_bt_oracle(calls, f, p, v, mc, ms)
        same_chains(calls, gus, gan, us, an)
    assert sum(len(u) for u in exp[0][2]) > 100


def test_oracle_vs_reference_live():
    lib = oracle_lib.ref_chain_bt()
    if lib is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    calls = gen.chain_dataset("small", num_calls=150, seed=91, median_n=500, max_n=12000)
    aq = [np.float32(int(((calls.y[calls.offsets[c]:calls.offsets[c + 1]] >> np.uint64(32)) & np.uint64(0xff)).sum()))
          / np.float32(calls.offsets[c + 1] - calls.offsets[c]) for c in range(calls.ncalls)]
    calls.avg_qspan = np.array(aq, np.float32)
    f, p, _, v, _ = oracle_lib.chain_oracle(calls)
    for mc, ms in [(3, 40), (1, 0)]:
        rus, ran = oracle_lib.ref_chain_bt_run(lib, calls, mc, ms)
        _, gus, gan = oracle_lib.chain_bt_oracle(calls, f, p, v, mc, ms)
        same_chains(calls, gus, gan, rus, ran)


def gpu_chains(b, calls):
    nch, u, nan, ax, ay, tc, ta = b.chains()
    us, an = [], []
    for c in range(calls.ncalls):
        o = int(calls.offsets[c])
        us.append(u[o:o + int(nch[c])])
        an.append((ax[2 * o:2 * o + int(nan[c])], ay[2 * o:2 * o + int(nan[c])]))
    assert tc == int(nch.sum()) and ta == int(nan.sum())
    return us, an


@pytest.mark.gpu
def test_gpu_vs_golden(golden):
    from genomicsbench_palisade_amd import chain, set_device
    set_device(0)
    calls, exp = golden
    b = chain.ChainBatch(calls)
    b.run()
    for mc, ms, us, an in exp:
        b.backtrack(mc, ms)
        gus, gan = gpu_chains(b, calls)
        same_chains(calls, gus, gan, us, an)
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,ncalls,median,maxn", [(3, 300, 1500, 87271), (4, 2000, 150, 3000)])
def test_gpu_vs_oracle(seed, ncalls, median, maxn):
    """Bench-shaped calls (one of 87 271 anchors) and many small ones; the DP outputs are the GPU's
    (bit-exact to the oracle's by test_chain.py)."""
    from genomicsbench_palisade_amd import chain, set_device
    set_device(0)
    calls = gen.chain_dataset("small", num_calls=ncalls, seed=seed, median_n=median, max_n=maxn)
    b = chain.ChainBatch(calls)
    b.run()
    f, p, _, v, _ = b.results()
    for mc, ms in [(3, 40), (1, 0)]:
        b.backtrack(mc, ms)
        gus, gan = gpu_chains(b, calls)
        _, ous, oan = oracle_lib.chain_bt_oracle(calls, f, p, v, mc, ms, 8)
        same_chains(calls, gus, gan, ous, oan)
    b.backtrack(3, 40)  # re-run on the same device buffers
    gus, gan = gpu_chains(b, calls)
    _, ous, oan = oracle_lib.chain_bt_oracle(calls, f, p, v, 3, 40, 8)
    same_chains(calls, gus, gan, ous, oan)
    b.close()


def twin_calls(seed, ncalls, n):
    """Every anchor twice, at the same x on two parallel diagonals (y and y + 2 000): chains come in
    pairs whose first anchors share x, so calls with more than 64 kept chains sort tied keys -- the
    path where k_reorder leaves its parallel sort to the replay of ksort (whose tie order is its own)."""
    rng = np.random.default_rng(seed)
    offs, xs, ys, aq = [0], [], [], []
    for _ in range(ncalls):
        x, y, a = gen.chain_call(rng, n)
        x2 = np.repeat(x, 2)
        y2 = np.repeat(y, 2)
        y2[1::2] += np.uint64(2000)
        xs.append(x2)
        ys.append(y2)
        aq.append(a)
        offs.append(offs[-1] + len(x2))
    params = np.tile(np.array([5000, 5000, 500, 1], np.int32), (ncalls, 1))
    return gen.ChainCalls(np.array(offs, np.int64), np.concatenate(xs), np.concatenate(ys), np.array(aq, np.float32),
                          params)


@pytest.mark.gpu
def test_gpu_tied_keys_vs_oracle():
    from genomicsbench_palisade_amd import chain, set_device
    set_device(0)
    calls = twin_calls(17, 40, 3000)
    b = chain.ChainBatch(calls)
    b.run()
    f, p, _, v, _ = b.results()
    for mc, ms in [(3, 40), (1, 0)]:
        b.backtrack(mc, ms)
        gus, gan = gpu_chains(b, calls)
        _, ous, oan = oracle_lib.chain_bt_oracle(calls, f, p, v, mc, ms, 8)
        same_chains(calls, gus, gan, ous, oan)
        assert max(len(u) for u in ous) > 64  # the sort path, not the 64-lane ranking
    b.close()
