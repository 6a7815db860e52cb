"""fmi search probe: a 128 Mbp synthetic index and 2M reads, timed search (for PMC / phase clocks)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genomicsbench_palisade_amd import fmi, gen, set_device
set_device(0)
mbp = float(os.environ.get("FMI_PROBE_MBP", "512"))
nreads = int(os.environ.get("FMI_PROBE_READS", "2000000"))
ref = gen.fmi_reference(int(mbp * 1e6), seed=7)
idx = fmi.Index.build(ref)
codes, lens = gen.fmi_reads(ref, nreads, read_len=151, seed=8)
rs = fmi.Reads(idx, codes, lens)
for _ in range(2):
    rs.search(19)
    rs.sync()
    a, b, calls = rs.timing()
    print(f"search {a:.2f} ms total {b:.2f} ms, {calls / nreads:.1f} ext/read, {nreads / a / 1e3:.2f} Mreads/s", flush=True)
