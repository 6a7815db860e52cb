"""computelikelihoodsboth per batch (the reference driver's granularity, PairHMMUnitTest.cpp:549-593) on the
'large' job: seconds for all 64 batches, the kernel-only rate of the same job, and (GB_PHMM_HOSTPROF
style) the host phases of a few calls."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import gen, phmm, set_device  # noqa: E402
from genomicsbench_palisade_amd._tc import TestcaseArray  # noqa: E402

set_device(0)
phmm.init_pairhmm()
batches = gen.phmm_dataset("large", 64, seed=1)
arrs = [TestcaseArray.from_batch(b) for b in batches]
outs = [np.zeros(max(a.n, 1)) for a in arrs]
cells = sum(a.cells() for a in arrs)
lib = ctypes.CDLL(os.path.join(ROOT, "genomicsbench_palisade_amd", "lib", "libgkl_pairhmm_c.so"))
both = getattr(lib, "_Z22computelikelihoodsbothP8testcasePdi")
both.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
full = phmm.DeviceBatch(TestcaseArray.from_batches(batches))
for _ in range(3):
    full.run()
full.sync()
t0 = time.perf_counter()
for _ in range(5):
    full.run()
full.sync()
kt = (time.perf_counter() - t0) / 5
full.close()
for rep in range(3):
    t0 = time.perf_counter()
    for a, o in zip(arrs, outs):
        both(ctypes.addressof(a.arr), o.ctypes.data, a.n)
    t = time.perf_counter() - t0
    print(f"per batch: {len(arrs)} calls, {t * 1e3:.1f} ms = {cells / t / 1e9:.1f} GCUPS "
          f"({kt / t:.3f} of the whole-job kernel rate {cells / kt / 1e9:.0f} GCUPS)", flush=True)
os.environ["GB_PHMM_HOSTPROF"] = "1"
for a, o in list(zip(arrs, outs))[:3]:
    print(f"-- batch of {a.n} testcases, {a.cells() / 1e6:.0f} M cells", file=sys.stderr, flush=True)
    both(ctypes.addressof(a.arr), o.ctypes.data, a.n)
