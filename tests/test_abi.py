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


def test_chain_rejects_oversized_call_before_touching_the_device():
    """A call must hold < 2^30 anchors (int32 indices, buffer-store offsets): GB_ERR_ARG, checked
    before any device work, so this runs without a GPU."""
    import ctypes
    import numpy as np
    from genomicsbench_palisade_amd import lib
    L = lib()
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    L.gb_chain_batch_create.argtypes = [i64, vp, vp, vp, vp, vp, ctypes.POINTER(vp)]
    offsets = np.array([0, 1 << 30], np.int64)
    aq = np.ones(1, np.float32)
    p4 = np.array([5000, 5000, 500, 1], np.int32)
    xy = np.zeros(1, np.uint64)  # never read: the size check comes first
    h = vp()
    rc = L.gb_chain_batch_create(1, offsets.ctypes.data, aq.ctypes.data, p4.ctypes.data, xy.ctypes.data,
                                 xy.ctypes.data, ctypes.byref(h))
    assert rc == -1 and not h.value  # GB_ERR_ARG, no batch


def test_pmc_summary_applies_calibrated_read_class_factors(tmp_path):
    """tools/pmc_summary.py: gather-class kernels keep FETCH_SIZE, stream-class kernels double it
    (profiles/r01g_pmc_calib.txt), WRITE_SIZE as measured; raw counters are kept."""
    import csv
    import json
    import subprocess
    import sys
    cols = ["Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]
    for what, counter, vals in [("fetch", "FETCH_SIZE", (100.0, 10.0)), ("write", "WRITE_SIZE", (7.0, 3.0))]:
        d = tmp_path / what
        d.mkdir()
        with open(d / "run_counter_collection.csv", "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=cols)
            w.writeheader()
            w.writerow({"Kernel_Name": "void gbfmi::smem_search<true>(gbfmi::SearchArgs)", "Counter_Name": counter,
                        "Counter_Value": vals[0], "Start_Timestamp": 0, "End_Timestamp": 1000000})
            w.writerow({"Kernel_Name": "void gbchain::chain_kernel<0>(gbchain::Args)", "Counter_Name": counter,
                        "Counter_Value": vals[1], "Start_Timestamp": 0, "End_Timestamp": 2000000})
    dst = tmp_path / "pmc.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(tmp_path / "fetch"),
                    str(tmp_path / "write"), str(dst)], check=True, capture_output=True)
    d = json.load(open(dst))
    assert d["smem_search"]["fetch_class"] == "gather" and d["smem_search"]["fetch_bytes"] == 100.0 * 1024
    assert d["chain_kernel"]["fetch_class"] == "stream" and d["chain_kernel"]["fetch_bytes"] == 2 * 10.0 * 1024
    assert d["chain_kernel"]["fetch_bytes_raw"] == 10.0 * 1024 and d["chain_kernel"]["write_bytes"] == 3.0 * 1024
