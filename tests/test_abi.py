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


@pytest.mark.parametrize("header", sorted(h for h in os.listdir(INC) if h.startswith("gb_")))
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


def test_no_device_is_reported_not_faked():
    import genomicsbench_palisade_amd as gb
    n = gb.device_count()
    if n == 0:
        with pytest.raises(gb.GbError):
            gb.set_device(0)
