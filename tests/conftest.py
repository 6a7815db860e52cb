import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")


def _split(data, lens):
    out, o = [], 0
    for n in lens:
        out.append(data[o:o + n].tobytes())
        o += int(n)
    return out


@pytest.fixture(scope="session")
def phmm_golden():
    """Golden vectors from the reference GKL kernels (tests/golden/make_golden.py)."""
    from genomicsbench_palisade_amd._tc import TestcaseArray
    z = np.load(os.path.join(GOLDEN, "phmm_golden.npz"))
    rl = z["read_len"]
    reads = list(zip(*[_split(z[k], rl) for k in ("read_bases", "read_q", "read_i", "read_d", "read_c")]))
    haps = _split(z["hap_bases"], z["hap_len"])
    prl = z["pair_read_len"]
    preads = list(zip(*[_split(z[k], prl) for k in ("pair_read_bases", "pair_read_q", "pair_read_i",
                                                     "pair_read_d", "pair_read_c")]))
    phaps = _split(z["pair_hap_bases"], z["pair_hap_len"])
    return {
        "cross": TestcaseArray(reads, haps),
        "cross_expect": (z["cross_final"], z["cross_raw_f"], z["cross_raw_d"]),
        "pairs": TestcaseArray.from_pairs(list(zip(preads, phaps))),
        "pairs_expect": (z["pair_final"], z["pair_raw_f"], z["pair_raw_d"]),
    }


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


def assert_phmm_exact(got, expect):
    """(results, raw f32, raw f64[, used_double]) of the HIP path against the reference's / the
    oracle's: bit-exact on everything computelikelihoodsboth exposes (phmm.parity_mismatches: raw f32
    where the reference's passes MIN_ACCEPTED, the reference's value or the early exit's 0 below it),
    and the same fallback choice."""
    from genomicsbench_palisade_amd.phmm import MIN_ACCEPTED, parity_mismatches
    got = tuple(np.ascontiguousarray(x) for x in got)
    expect = tuple(np.ascontiguousarray(x) for x in expect)
    bad = parity_mismatches(got, expect)
    assert not (bad["log10"] or bad["raw_f32"] or bad["raw_f64"]), bad
    if len(got) > 3:
        assert (got[3].astype(bool) == (expect[1] < MIN_ACCEPTED)).all(), "fallback choice differs"
    return bad


def gpu_available():
    try:
        import genomicsbench_palisade_amd as gb
        return gb.device_count() > 0
    except Exception:
        return False
