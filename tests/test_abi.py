"""CPU: libgb.so / libgkl_pairhmm_c.so load and export every symbol the public headers declare."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

INC = os.path.join(ROOT, "include")
LIB = os.path.join(ROOT, "genomicsbench_palisade_amd", "lib")


def declared(header):
    src = open(os.path.join(INC, header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(gb_\w+)\s*\(", src, flags=re.M)))


@pytest.mark.parametrize("header", sorted(h for h in os.listdir(INC) if h.startswith("gb_") and h.endswith(".h")))
def test_libgb_exports_header(header):
    lib = ctypes.CDLL(os.path.join(LIB, "libgb.so"))
    names = declared(header)
    assert names, header
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"{header}: not exported: {missing}"


def test_dropin_exports_reference_symbols():
    lib = ctypes.CDLL(os.path.join(LIB, "libgkl_pairhmm_c.so"))
    for sym in ("_Z11initPairHMMv", "_Z22computelikelihoodsbothP8testcasePdi",
                "_Z23computelikelihoodsfloatP8testcasePf", "_Z24computelikelihoodsdoubleP8testcasePd"):
        assert hasattr(lib, sym), sym


CHAIN_SYM = "_Z17host_chain_kernelRSt6vectorI6call_tSaIS0_EERS_I8return_tSaIS4_EEi"
BSW_SYMS = ("_ZN16BandedPairWiseSWC1EiiiiiiPKaaai", "_ZN16BandedPairWiseSW11getScores16EP10dnaSeqPairPhS2_iti",
            "_ZN16BandedPairWiseSW10getScores8EP10dnaSeqPairPhS2_iti",
            "_ZN16BandedPairWiseSW15scalarBandedSWAEiPKhiS1_iiPiS2_S2_S2_S2_", "_ZN16BandedPairWiseSW8getTicksEv")


def test_chain_bsw_dropins_export_reference_symbols():
    """C++ linkage names a reference object file compiled against the reference headers binds to."""
    lib = ctypes.CDLL(os.path.join(LIB, "libgb_chain_dropin.so"))
    assert hasattr(lib, CHAIN_SYM)
    lib = ctypes.CDLL(os.path.join(LIB, "libgb_bsw_dropin.so"))
    for sym in BSW_SYMS:
        assert hasattr(lib, sym), sym


def test_chain_symbol_matches_reference_build():
    """The reference's own scalar host_kernel.cpp (oracle/_ref) exports the same mangled name."""
    import subprocess
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_chain.so")
    if not os.path.exists(ref):
        pytest.skip("oracle/_ref not built")
    out = subprocess.run(["nm", "-D", "--defined-only", ref], capture_output=True, text=True).stdout
    assert CHAIN_SYM in out


def test_no_device_is_reported_not_faked():
    import genomicsbench_palisade_amd as gb
    n = gb.device_count()
    if n == 0:
        with pytest.raises(gb.GbError):
            gb.set_device(0)
