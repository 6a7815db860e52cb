"""Estimate (CPU, f64 numpy) of the f32 work an exact early exit could skip in phmm: a testcase whose
probability mass crossing from row r to r+1 (sum over columns of z + w, the records the f32 kernel
already hands down) is below MIN_ACCEPTED / 2 must fail the f32 test (everything after the cut is
that mass times transitions and emissions <= 1), so its remaining f32 rows are wasted. 300 random
testcases of the bench's large job (seed 1)."""
import sys, numpy as np
sys.path.insert(0, '/root/repo')
from genomicsbench_palisade_amd import gen
batches = gen.phmm_dataset("large", 64, seed=1)
rng = np.random.default_rng(0)
# GKL tables (Context.h): ph2pr(q) = 10^(-q/10)
def ph2pr(q): return 10.0 ** (-np.asarray(q, np.float64) / 10.0)
tot_cells = 0; fail_cells = 0; saved_cells = 0; nfail = 0; n = 0
samples = []
for b in batches:
    for r in b.reads:
        for h in b.haps:
            samples.append((r, h))
idx = rng.choice(len(samples), 300, replace=False)
for k in idx:
    (bases, q, ii, dd, cc), hap = samples[k]
    R, C = len(bases), len(hap)
    rb = np.frombuffer(bases, np.uint8); hb = np.frombuffer(hap, np.uint8)
    q = np.frombuffer(q, np.uint8).astype(float); ii = np.frombuffer(ii, np.uint8).astype(float)
    dd = np.frombuffer(dd, np.uint8).astype(float); cc = np.frombuffer(cc, np.uint8).astype(float)
    pMX = ph2pr(ii); pMY = ph2pr(dd); pXX = ph2pr(cc); pYY = ph2pr(cc); pGAPM = 1 - pXX
    pMM = 1 - (pMX + pMY)
    err = ph2pr(q)
    init = 2.0 ** 120 / C
    Mp = np.zeros(C + 1); Xp = np.zeros(C + 1); Yp = np.full(C + 1, init); Yp[0] = 0  # row 0: Y = init (cols 1..C)
    Mp[:] = 0
    exit_row = None
    for r in range(R):
        match = (hb == rb[r]) | (rb[r] == ord('N')) | (hb == ord('N'))
        dist = np.where(match, 1 - err[r], err[r] / 3)
        M = np.zeros(C + 1); X = np.zeros(C + 1); Y = np.zeros(C + 1)
        prev_mm = pMM[r - 1] if r > 0 else 1.0  # transitions of row r applied to row r-1 values (GKL uses row r's)
        M[1:] = dist * (Mp[:-1] * pMM[r] + Xp[:-1] * pGAPM[r] + Yp[:-1] * pGAPM[r])
        X[1:] = Mp[1:] * pMX[r] + Xp[1:] * pXX[r]
        for c in range(1, C + 1):
            Y[c] = M[c - 1] * pMY[r] + Y[c - 1] * pYY[r]
        Mp, Xp, Yp = M, X, Y
        if r < R - 1 and exit_row is None:
            cross = (M[1:] * (pMM[r + 1] + pMX[r + 1]) + X[1:] * (pGAPM[r + 1] + pXX[r + 1]) + Y[1:] * pGAPM[r + 1]).sum()
            if cross < 0.5e-28:
                exit_row = r + 1
    res = M[1:].sum() + X[1:].sum()
    n += 1; tot_cells += R * C
    if res < 1e-28:
        nfail += 1; fail_cells += R * C
        if exit_row is not None:
            saved_cells += (R - exit_row) * C
print(f"sample {n}: failing {nfail} ({fail_cells/tot_cells:.3f} of cells); rows after the bound crossing {saved_cells/tot_cells:.3f} of all cells, {saved_cells/max(fail_cells,1):.3f} of failing cells")
