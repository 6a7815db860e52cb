import sys, os, time, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
from genomicsbench_palisade_amd import gen
from genomicsbench_palisade_amd._tc import TestcaseArray
import oracle_lib
ref = oracle_lib.ref_phmm(); o = oracle_lib.oracle()
print("avx512", ref.ref_phmm_has_avx512(), "affinity", len(os.sched_getaffinity(0)))
ta = TestcaseArray.from_batches(gen.phmm_dataset("large", 2, seed=1))
sub = ta.subset(np.arange(4000)); n = sub.n
eo, ef, ed = np.zeros(n), np.zeros(n, np.float32), np.zeros(n)
t = time.perf_counter(); o.phmm_oracle_batch(ctypes.addressof(sub.arr), n, eo.ctypes.data, ef.ctypes.data, ed.ctypes.data, None, 16); print("oracle16", time.perf_counter()-t, sub.cells()/(time.perf_counter()-t)/1e9)
for eng in (512, 256):
  for th in (1, 16):
    out, rf, rd = np.zeros(n), np.zeros(n, np.float32), np.zeros(n)
    t = time.perf_counter()
    ref.ref_phmm_batch(ctypes.addressof(sub.arr), n, out.ctypes.data, rf.ctypes.data, rd.ctypes.data, eng, th)
    dt = time.perf_counter() - t
    print(eng, th, round(dt, 3), "GCUPS", round(sub.cells() / dt / 1e9, 3), "exact", bool((out.view(np.uint64) == eo.view(np.uint64)).all()))
