"""Stale-LDS A/B: tests/test_lds_poison.py's chain check run against another build of libgb.so
(GB_LIB, e.g. tools/_ab/libgb_pre1da81ef.so: the current library with chain_rows.o built from the
commit before 1da81ef, whose stamp ring was not cleared at block start). Prints, per LDS pattern and
verification mode, how many anchors differ from the oracle -- the test must fail on that build.
    GB_LIB=tools/_ab/libgb_pre1da81ef.so python tools/lds_poison_ab.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import genomicsbench_palisade_amd as g  # noqa: E402
if os.environ.get("GB_LIB"):
    g.LIBGB = os.path.abspath(os.environ["GB_LIB"])
import oracle_lib  # noqa: E402
from genomicsbench_palisade_amd import chain, gen, set_device  # noqa: E402
from test_lds_poison import CHAIN_NAMES, PATTERNS  # noqa: E402

set_device(0)
pl = ctypes.CDLL(os.path.join(ROOT, "tests", "_build", "liblds_poison.so"))
pl.lds_poison.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
calls = gen.chain_dataset("small", num_calls=400, seed=21, median_n=1500, max_n=40000)
exp = oracle_lib.chain_oracle(calls, 8)
lib = os.path.basename(g.LIBGB)
fails = 0
for vlanes in ("1", "0"):
    os.environ["GB_CHAIN_VLANES"] = vlanes
    b = chain.ChainBatch(calls)
    for mode, value in [(None, None)] + PATTERNS:
        if mode is not None:
            assert pl.lds_poison(0, mode, value, 1) == 0
        b.run()
        got = b.results()
        bad = {name: int((got[k] != exp[k]).sum()) for k, name in enumerate(CHAIN_NAMES)}
        vis = got[4] - exp[4]
        ok = not any(bad.values()) and vis == 0
        fails += not ok
        print(f"{lib} GB_CHAIN_VLANES={vlanes} pattern {'none' if mode is None else (mode, value)}: "
              f"mismatches {bad}, visited {got[4]} vs {exp[4]} -> {'exact' if ok else 'WRONG'}", flush=True)
    b.close()
print(f"{lib}: {fails} wrong runs")
