"""Development probe: build a > 2^32-row index with a given GB_FMI_BUILD_CHUNK and report where the
CP_OCC invariants break (rows without a base, duplicate sampled SA values)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import fmi, gen, set_device  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 2_200_000_000
set_device(0)
t0 = time.time()
ref = gen.fmi_reference(G, seed=31, repeat_frac=0.001)
ref[G // 2:G // 2 + 20_000] = 0
idx = fmi.Index.build(ref)
print(f"chunk={os.environ.get('GB_FMI_BUILD_CHUNK', '')} build done {time.time() - t0:.1f}s", flush=True)
n, c5, sent = idx.info()
cp = idx.cp_occ()
oh = cp[:, 4:].view(np.uint64)
per = np.bitwise_count(oh).astype(np.int64).sum(axis=1)
full = np.full(len(cp), 64, np.int64)
full[-1] = n - (len(cp) - 1) * 64
full[sent >> 6] -= 1
bad = np.nonzero(per != full)[0]
print("n", n, "sentinel", sent, "bad blocks", len(bad), "first", bad[:10], "last", bad[-10:] if len(bad) else [],
      "missing rows", int((full - per)[bad].sum()) if len(bad) else 0, flush=True)
if len(bad):
    rows = bad * 64
    print("bad block rows / 2^30:", np.unique(rows >> 30), flush=True)
