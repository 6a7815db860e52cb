"""fmi hand-over probe: search time of one read set per (GB_FMI_HEAVY, GB_FMI_DRAIN, GB_FMI_HELP)
setting -- budget 1 hands every read over at once, so the wave-per-read routine does the whole set,
inside smem_search (help 1) or in smem_heavy after it (help 0)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import fmi, gen, set_device  # noqa: E402

set_device(0)
mbp = float(os.environ.get("FMI_PROBE_MBP", "64"))
nreads = int(os.environ.get("FMI_PROBE_READS", "200000"))
ref = gen.fmi_reference(int(mbp * 1e6), seed=7)
idx = fmi.Index.build(ref)
codes, lens = gen.fmi_reads(ref, nreads, read_len=151, seed=8)
rs = fmi.Reads(idx, codes, lens)
base = None
for v in os.environ.get("FMI_PROBE_SET", "1,0,0;1,0,1;2000,0,0;2000,0,1;2000,4,1;2000,4,0").split(";"):
    b, d, h = v.split(",")
    os.environ.update(GB_FMI_HEAVY=b, GB_FMI_DRAIN=d, GB_FMI_HELP=h)
    rs.search(19)
    rs.sync()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        rs.search(19)
        rs.sync()
        ts.append(time.perf_counter() - t0)
    a, tot, calls = rs.timing()
    sm = rs.results(batch_size=512)[0]
    same = "" if base is None else (" same SMEMs" if (sm == base).all() else " SMEMs DIFFER")
    if base is None:
        base = sm
    print(f"budget {b:>5} drain {d} help {h}: search {a:8.2f} ms (wall {min(ts) * 1e3:8.2f}), {calls / nreads:.1f} ext/read{same}",
          flush=True)
rs.close()
