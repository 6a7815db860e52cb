"""fmi A/B probe: the full 'large' read set and its 8 strong-scaling shards searched under each
setting of FMI_AB (';'-separated env assignments 'K=V,K=V'), interleaved over FMI_AB_REPS rounds on
the same index and reads, so box-to-box speed differences cancel. Per setting: full-set ms (min of
3 per round), worst shard ms (max over ranks of min of 3), and the shard ratio (full / 8 / worst)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import fmi, gen, set_device, shard  # noqa: E402

set_device(0)
nreads = int(os.environ.get("FMI_PROBE_READS", "10000000"))
ref = gen.fmi_reference(int(float(os.environ.get("FMI_PROBE_MBP", "512")) * 1e6), seed=7)
idx = fmi.Index.build(ref)
codes, lens = gen.fmi_reads(ref, nreads, read_len=151, seed=8)
full = fmi.Reads(idx, codes, lens)
shards = []
for r in range(8):
    lo, hi = shard.read_range(nreads, r, 8)
    shards.append(fmi.Reads(idx, codes[lo:hi], lens[lo:hi]))
sets = [s for s in os.environ.get("FMI_AB", "GB_FMI_LIST=0;GB_FMI_LIST=32").split(";")]
keys = sorted({kv.split("=")[0] for s in sets for kv in s.split(",") if kv})


def timed(rs, n=3):
    rs.search(19)
    rs.sync()
    best = 1e9
    for _ in range(n):
        t0 = time.perf_counter()
        rs.search(19)
        rs.sync()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


res = {s: [] for s in sets}
for rep in range(int(os.environ.get("FMI_AB_REPS", "3"))):
    for s in sets:
        for k in keys:
            os.environ.pop(k, None)
        for kv in s.split(","):
            if kv:
                k, v = kv.split("=")
                os.environ[k] = v
        f = timed(full)
        w = max(timed(rs) for rs in shards)
        res[s].append((f, w))
        print(f"rep {rep} [{s}]: full {f:7.2f} ms ({nreads / f / 1e3:.2f} Mreads/s), worst shard {w:6.2f} ms, "
              f"ratio {f / 8 / w:.4f}", flush=True)
print("summary (median over rounds):")
for s in sets:
    a = np.array(res[s])
    f, w = np.median(a[:, 0]), np.median(a[:, 1])
    print(f"  [{s}]: full {f:7.2f} ms = {nreads / f / 1e3:.2f} Mreads/s; worst shard {w:6.2f} ms; ratio {f / 8 / w:.4f}",
          flush=True)
