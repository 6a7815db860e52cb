"""First-call costs of the phmm drop-in in a fresh process: gb_phmm_init (initPairHMM) timed, then
gb_phmm_compute (computelikelihoodsboth's C ABI) over the 'large' job three times, each timed; with
GB_PHMM_HOSTPROF=1 the library prints its host phases. The gap between call 1 and call 3 is what a
cold process (bin/phmm) pays inside the reference's timed region.
    python tools/phmm_cold_probe.py
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import gen, lib, set_device  # noqa: E402
from genomicsbench_palisade_amd._tc import TestcaseArray  # noqa: E402

ta = TestcaseArray.from_batches(gen.phmm_dataset("large", int(os.environ.get("PHMM_BATCHES", "64")), seed=1))
cells = ta.cells()
L = lib()
set_device(0)
t0 = time.perf_counter()
assert L.gb_phmm_init() == 0
print(f"init {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
out = np.zeros(ta.n)
for k in range(3):
    t0 = time.perf_counter()
    assert L.gb_phmm_compute(ctypes.addressof(ta.arr), ta.n, out.ctypes.data, None, None, None) == 0
    t = time.perf_counter() - t0
    print(f"compute call {k + 1}: {1e3 * t:.1f} ms ({cells / t / 1e9:.0f} GCUPS)", flush=True)
