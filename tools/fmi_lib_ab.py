"""fmi library A/B: the full 'large' read set and its shard 0 of 8 searched with the libgb.so named
by FMI_LIB (default: the tree's own), so two builds can be timed alternately on one box."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import genomicsbench_palisade_amd as g  # noqa: E402

if os.environ.get("FMI_LIB"):
    g.LIBGB = os.path.abspath(os.environ["FMI_LIB"])
from genomicsbench_palisade_amd import fmi, gen, set_device, shard  # noqa: E402

set_device(0)
nreads = int(os.environ.get("FMI_PROBE_READS", "10000000"))
ref = gen.fmi_reference(512_000_000, seed=7)
idx = fmi.Index.build(ref)
codes, lens = gen.fmi_reads(ref, nreads, read_len=151, seed=8)
lo, hi = shard.read_range(nreads, 0, 8)
out = []
for name, (a, b) in (("full", (0, nreads)), ("shard0", (lo, hi))):
    rs = fmi.Reads(idx, codes[a:b], lens[a:b])
    rs.search(19)
    rs.sync()
    best, kbest = 1e9, 1e9
    for _ in range(4):
        t0 = time.perf_counter()
        rs.search(19)
        rs.sync()
        best = min(best, time.perf_counter() - t0)
        kbest = min(kbest, rs.timing()[0])
    rs.close()
    out.append(f"{name} wall {best * 1e3:.2f} ms, search {kbest:.2f} ms ({(b - a) / best / 1e6:.2f} Mreads/s)")
print(f"[{os.path.basename(os.path.dirname(os.path.dirname(g.LIBGB)))}/{os.path.basename(g.LIBGB)}] " + "; ".join(out),
      flush=True)
