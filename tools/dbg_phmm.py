import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import conftest, oracle_lib
from genomicsbench_palisade_amd import phmm, set_device
set_device(0); phmm.init_pairhmm()
g = conftest.phmm_golden.__wrapped__()
ta = g["cross"]; e_out, e_rf, e_rd = g["cross_expect"]
res, rf, rd, ud = phmm.compute_likelihoods_both(ta)
bad = np.nonzero(rd.view(np.uint64) != e_rd.view(np.uint64))[0]
print("nbad", len(bad), "of", ta.n, "fallbacks exp", (e_rf < np.float32(1e-28)).sum(), "got", ud.sum())
for k in bad[:12]:
    t = ta.np_arr[k]
    print(k, "R", t["rslen"], "C", t["haplen"], "rf", rf[k], e_rf[k], "rd", rd[k], e_rd[k], "ud", ud[k])
rdall = phmm.compute_f64(ta)
o = oracle_lib.oracle()
exp = np.array([o.phmm_oracle_prob_f64(ctypes.addressof(ta.arr[k])) for k in range(ta.n)])
b2 = np.nonzero(rdall.view(np.uint64) != exp.view(np.uint64))[0]
print("f64-all mismatches", len(b2))
for k in b2[:12]:
    t = ta.np_arr[k]
    print(k, "R", t["rslen"], "C", t["haplen"], rdall[k], exp[k], rdall[k]/exp[k])
