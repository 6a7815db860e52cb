"""computelikelihoodsboth once per batch over the 'large' job (the reference's call pattern,
PairHMMUnitTest.cpp:549-593): per call wall time against its cells, the total, and the calls' share
of fixed cost (time of calls under 0.2 G cells). PHMM_PERBATCH_CONFIGS: ';'-separated env settings
(VAR=VALUE joined by '+'), each timed in this process (the knobs are read per call).
    python tools/phmm_perbatch_probe.py
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import gen, set_device  # noqa: E402
from genomicsbench_palisade_amd._tc import TestcaseArray  # noqa: E402

set_device(0)
lib = ctypes.CDLL(os.path.join(ROOT, "genomicsbench_palisade_amd", "lib", "libgkl_pairhmm_c.so"))
lib._Z11initPairHMMv()
both = lib._Z22computelikelihoodsbothP8testcasePdi
both.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
batches = gen.phmm_dataset("large", int(os.environ.get("PHMM_BATCHES", "64")), seed=1)
arrs = [TestcaseArray.from_batch(b) for b in batches]
outs = [np.zeros(max(a.n, 1)) for a in arrs]
cells = np.array([a.cells() for a in arrs], np.float64)
for cfg in os.environ.get("PHMM_PERBATCH_CONFIGS", "").split(";"):
    for k in [k for k in os.environ if k.startswith("GB_PHMM")]:
        os.environ.pop(k)
    for kv in [c for c in cfg.split("+") if c]:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    for a, o in zip(arrs, outs):  # warm
        both(ctypes.addressof(a.arr), o.ctypes.data, a.n)
    best = None
    for rep in range(3):
        ts = []
        for a, o in zip(arrs, outs):
            t0 = time.perf_counter()
            both(ctypes.addressof(a.arr), o.ctypes.data, a.n)
            ts.append(time.perf_counter() - t0)
        ts = np.array(ts)
        if best is None or ts.sum() < best.sum():
            best = ts
    small = cells < 0.2e9
    print(f"[{cfg or 'default':30s}] total {best.sum() * 1e3:7.2f} ms ({cells.sum() / best.sum() / 1e9:6.1f} GCUPS); "
          f"{int(small.sum())} calls < 0.2 G cells: {best[small].sum() * 1e3:6.2f} ms "
          f"({best[small].mean() * 1e3:.3f} ms each, {cells[small].sum() / 1e9:.2f} G cells); "
          f"largest call {cells.max() / 1e9:.2f} G cells {best[cells.argmax()] * 1e3:.2f} ms; "
          f"min call {best.min() * 1e3:.3f} ms", flush=True)
    big = np.argsort(-cells)[:6]
    print("   biggest calls (G cells, ms, GCUPS): " + ", ".join(
        f"{cells[i] / 1e9:.2f}/{best[i] * 1e3:.2f}/{cells[i] / best[i] / 1e9:.0f}" for i in big), flush=True)
