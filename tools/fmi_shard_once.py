"""Search the bench's fmi 'large' 1/8 shard (or FMI_PROBE_READS reads) a few times: a short run to put
under rocprofv3 --kernel-trace (the knobs come from the environment)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import fmi, gen, set_device, shard  # noqa: E402

set_device(0)
nreads = int(os.environ.get("FMI_PROBE_READS", "10000000"))
ref = gen.fmi_reference(512_000_000, seed=7)
idx = fmi.Index.build(ref)
codes, lens = gen.fmi_reads(ref, nreads, read_len=151, seed=8)
lo, hi = shard.read_range(nreads, 0, int(os.environ.get("FMI_OF", "8")))
rs = fmi.Reads(idx, codes[lo:hi], lens[lo:hi])
for _ in range(int(os.environ.get("FMI_REPS", "3"))):
    t0 = time.perf_counter()
    rs.search(19)
    rs.sync()
    print(f"search {(time.perf_counter() - t0) * 1e3:.2f} ms, ctl {rs.ctl().tolist()}", flush=True)
rs.close()
