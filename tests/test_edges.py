"""Edge cases the benchmark shapes never produce, for the phmm and chain paths: empty batches,
minimal and stripe-boundary shapes, the haplotype-length cap, arbitrary q/i/d/c bytes (the
reference indexes its tables with `& 127`, Context.h / avx-pairhmm-template.h:83-128), non-ACGTN
bases (ConvertChar maps them to A), and chain calls with 0/1/2 anchors, duplicates, mixed
strands/references, split-read segments (n_segs > 1, host_kernel.cpp:47-66) and degenerate
windows. CPU: the oracle against the reference builds (oracle/_ref, skipped when absent). GPU:
the HIP kernels against the oracle, bit-exact."""
import ctypes

import numpy as np
import pytest

import oracle_lib
from conftest import assert_phmm_exact, bits
from genomicsbench_palisade_amd import gen
from genomicsbench_palisade_amd._tc import TestcaseArray

# ---------------------------------------------------------------------------------------------
# phmm

ALPHABET = np.frombuffer(b"ACGTNacgtnRYX-", np.uint8)


def phmm_edge_cases(seed=0):
    rng = np.random.default_rng(seed)
    pairs = []
    for rl in (1, 2, 63, 64, 65, 127, 128, 129, 250):
        for hl in (1, 2, 64, 473, 4096):
            if rl * hl > 250 * 1200 and rl > 65:  # keep the oracle's share of the test short
                continue
            src = rng.choice(ALPHABET[:4], size=max(rl, hl) + 8)
            hap = src[:hl].copy()
            rd = src[:rl].copy()
            odd = rng.random(rl) < 0.05
            rd[odd] = rng.choice(ALPHABET, size=int(odd.sum()))
            oddh = rng.random(hl) < 0.02
            hap[oddh] = rng.choice(ALPHABET, size=int(oddh.sum()))
            # q/i/d/c: the benchmark's ranges for most cases, any byte for a third of them
            if rng.random() < 0.33:
                q, i, d, c = (rng.integers(0, 256, rl).astype(np.uint8) for _ in range(4))
            else:
                q = rng.integers(6, 41, rl).astype(np.uint8)
                i = rng.integers(40, 46, rl).astype(np.uint8)
                d = rng.integers(40, 46, rl).astype(np.uint8)
                c = np.full(rl, 10, np.uint8)
            pairs.append(((rd.tobytes(), q.tobytes(), i.tobytes(), d.tobytes(), c.tobytes()), hap.tobytes()))
    # an all-N read and a read against an all-N haplotype
    n40 = b"N" * 40
    qs = bytes([30] * 40), bytes([45] * 40), bytes([45] * 40), bytes([10] * 40)
    pairs.append(((n40,) + qs, b"ACGT" * 30))
    pairs.append(((b"ACGT" * 10,) + qs, b"N" * 120))
    return TestcaseArray.from_pairs(pairs)


def phmm_oracle(ta):
    o = oracle_lib.oracle()
    n = ta.n
    out, rf, rd = np.zeros(n), np.zeros(n, np.float32), np.zeros(n)
    ud = np.zeros(n, np.int32)
    o.phmm_oracle_batch(ctypes.addressof(ta.arr), n, out.ctypes.data, rf.ctypes.data, rd.ctypes.data,
                        ud.ctypes.data, 8)
    return out, rf, rd


def test_phmm_edge_oracle_vs_reference_live():
    """The reference GKL kernels (AVX2 and AVX-512 engines) on the edge set: raw f32, raw f64 and
    final results identical to the oracle's."""
    ref = oracle_lib.ref_phmm()
    if ref is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    ta = phmm_edge_cases()
    got = phmm_oracle(ta)
    for eng in (256, 512):
        exp = np.zeros(ta.n), np.zeros(ta.n, np.float32), np.zeros(ta.n)
        ref.ref_phmm_batch(ctypes.addressof(ta.arr), ta.n, exp[0].ctypes.data, exp[1].ctypes.data,
                           exp[2].ctypes.data, eng, 4)
        for k in range(3):
            assert (bits(got[k]) == bits(exp[k])).all(), (eng, k)


@pytest.mark.gpu
def test_phmm_gpu_edges_bit_exact():
    from genomicsbench_palisade_amd import phmm, set_device
    set_device(0)
    phmm.init_pairhmm()
    ta = phmm_edge_cases()
    got = phmm.compute_likelihoods_both(ta)
    exp = phmm_oracle(ta)
    assert_phmm_exact(got, exp)


@pytest.mark.gpu
def test_phmm_gpu_longest_haplotype():
    """Haplotypes up to 9400 columns keep their stack's boundary records in LDS (the f64 pass: 17 bytes
    per column); longer ones -- 9401, 20000 and the 65535 maximum of the 16-bit descriptor field --
    run on the kLong kernels (records in global scratch), bit-exact against the oracle in both
    passes, in one batch beside ordinary stacks; 65536 is refused with GB_ERR_ARG (the GKL drop-in
    then aborts, as documented in include/gb_phmm.h)."""
    from genomicsbench_palisade_amd import GbError, phmm, set_device
    set_device(0)
    phmm.init_pairhmm()
    rng = np.random.default_rng(11)
    src = rng.choice(ALPHABET[:4], size=65536)
    qs = tuple(bytes(v) for v in ([30] * 12, [45] * 12, [45] * 12, [10] * 12))
    q40 = tuple(bytes(v) for v in ([40] * 150, [45] * 150, [45] * 150, [10] * 150))
    pairs = []
    for hl in (300, 9400, 9401, 20000, 65535):
        for st in (hl // 3, hl - 12):
            pairs.append(((src[st:st + 12].tobytes(),) + qs, src[:hl].tobytes()))
            # a random 150-base read at Q40: far below 1e-28 in f32, so the f64 pass runs it
            pairs.append(((rng.choice(ALPHABET[:4], size=150).tobytes(),) + q40, src[:hl].tobytes()))
    ok = TestcaseArray.from_pairs(pairs)
    got = phmm.compute_likelihoods_both(ok)
    exp = phmm_oracle(ok)
    assert (exp[1] < 1e-28).any() and (exp[1] >= 1e-28).any()  # both passes exercised
    assert_phmm_exact(got, exp)
    too_long = TestcaseArray.from_pairs([((src[:12].tobytes(),) + qs, (src.tobytes() * 2)[:65536])])
    with pytest.raises(GbError):
        phmm.compute_likelihoods_both(too_long)


@pytest.mark.gpu
def test_phmm_gpu_empty_batch():
    from genomicsbench_palisade_amd import phmm, set_device
    set_device(0)
    phmm.init_pairhmm()
    ta = TestcaseArray.from_pairs([])
    out = phmm.compute_likelihoods_both(ta)
    assert all(len(o) == 0 for o in out[:3])


# ---------------------------------------------------------------------------------------------
# chain


def chain_edge_calls(seed=3):
    rng = np.random.default_rng(seed)
    calls = []  # (x, y, avg_qspan, params4)

    def add(x, y, aq=18.0, p=(5000, 5000, 500, 1)):
        calls.append((np.asarray(x, np.uint64), np.asarray(y, np.uint64), aq, p))

    add([], [])                                                   # empty call
    add([(3 << 32) | 1000], [(19 << 32) | 5])                     # one anchor
    add([(3 << 32) | 1000] * 2, [(19 << 32) | 5] * 2)             # duplicate anchors
    x, y, aq = gen.chain_call(rng, 600)
    add(x, y, aq)                                                 # an ordinary call between edge ones
    add([], [])
    # mixed strands / references in one call, anchors sorted by x
    xs = np.sort((rng.integers(0, 2, 400).astype(np.uint64) << np.uint64(63)) |
                 (rng.integers(0, 3, 400).astype(np.uint64) << np.uint64(32)) |
                 rng.integers(0, 4000, 400).astype(np.uint64))
    ys = (np.uint64(15) << np.uint64(32)) | rng.integers(0, 3000, 400).astype(np.uint64)
    add(xs, ys, 15.0)
    # degenerate windows: max_dist 1, band 0
    x, y, aq = gen.chain_call(rng, 500)
    add(x, y, aq, (1, 1, 0, 1))
    # split-read segments: seg ids 0..2 in y bits 48+, n_segs 3 (different-segment gap rule)
    x, y, aq = gen.chain_call(rng, 1500)
    seg = rng.integers(0, 3, len(y)).astype(np.uint64)
    add(x, y | (seg << np.uint64(48)), aq, (5000, 300, 500, 3))
    # span 0 / 255 anchors and an extreme avg_qspan
    x, y, _ = gen.chain_call(rng, 800)
    sp = rng.choice(np.array([0, 1, 255], np.uint64), len(y))
    add(x, (y & np.uint64(0xFFFFFFFF)) | (sp << np.uint64(32)), 4000.0)
    # all anchors at one reference position (every pair has dr == 0)
    add(np.full(300, (5 << 32) | 77, np.uint64), (np.uint64(19) << np.uint64(32)) | np.arange(300, dtype=np.uint64), 19.0)
    offs = np.zeros(len(calls) + 1, np.int64)
    offs[1:] = np.cumsum([len(c[0]) for c in calls])
    return gen.ChainCalls(offs, np.concatenate([c[0] for c in calls]), np.concatenate([c[1] for c in calls]),
                          np.array([c[2] for c in calls], np.float32), np.array([c[3] for c in calls], np.int32))


NAMES = ["scores", "parents", "targets", "peak_scores"]


def assert_chain_same(got, exp):
    for k, name in enumerate(NAMES):
        bad = np.nonzero(got[k] != exp[k])[0]
        assert len(bad) == 0, f"{name}: {len(bad)} mismatches, first at {bad[:5]}"


def test_chain_edge_oracle_vs_reference_live():
    lib = oracle_lib.ref_chain()
    if lib is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    calls = chain_edge_calls()
    assert_chain_same(oracle_lib.chain_oracle(calls), oracle_lib.ref_chain_run(lib, calls))


@pytest.mark.gpu
def test_chain_gpu_edges_bit_exact():
    from genomicsbench_palisade_amd import chain, set_device
    set_device(0)
    calls = chain_edge_calls()
    exp = oracle_lib.chain_oracle(calls)
    b = chain.ChainBatch(calls)
    b.run()
    got = b.results()
    assert_chain_same(got, exp)
    assert got[4] == exp[4]  # visited (i, j) pairs
    from test_chain_bt import gpu_chains, same_chains
    f, p, _, v, _ = exp
    for mc, ms in ((1, 0), (3, 40)):
        b.backtrack(mc, ms)
        gus, gan = gpu_chains(b, calls)
        _, ous, oan = oracle_lib.chain_bt_oracle(calls, f, p, v, mc, ms)
        same_chains(calls, gus, gan, ous, oan)
    b.close()


@pytest.mark.gpu
def test_chain_gpu_no_calls():
    from genomicsbench_palisade_amd import chain, set_device
    set_device(0)
    calls = gen.ChainCalls(np.zeros(1, np.int64), np.zeros(0, np.uint64), np.zeros(0, np.uint64),
                           np.zeros(0, np.float32), np.zeros((0, 4), np.int32))
    b = chain.ChainBatch(calls)
    b.run()
    got = b.results()
    assert all(len(g) == 0 for g in got[:4])
    b.close()
