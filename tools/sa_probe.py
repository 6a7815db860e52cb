"""SA-lookup probe: 512 Mbp synthetic index, 2M reads searched, then get_sa_entries_prefetch over every
SMEM with launch-shape sweeps (GB_SA_BLOCKS_PER_CU is read at every launch)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genomicsbench_palisade_amd import fmi, gen, set_device
set_device(0)
mbp = float(os.environ.get("FMI_PROBE_MBP", "512"))
nreads = int(os.environ.get("FMI_PROBE_READS", "2000000"))
ref = gen.fmi_reference(int(mbp * 1e6), seed=7)
idx = fmi.Index.build(ref)
codes, lens = gen.fmi_reads(ref, nreads, read_len=151, seed=8)
rs = fmi.Reads(idx, codes, lens)
rs.search(19)
rs.sync()
for bpc in os.environ.get("SA_PROBE_BPC", "2,4,8,16").split(","):
    os.environ["GB_SA_BLOCKS_PER_CU"] = bpc
    best = 1e9
    for _ in range(4):
        rs.sa_run(500, fmi.SA_PREFETCH)
        rs.sync()
        ms, steps, nc = rs.sa_timing()
        best = min(best, ms)
    gbs = (steps * 64 + nc * 24) / (best * 1e-3) / 1e9
    print(f"blocks/CU {bpc}: {best:.3f} ms, {nc / best / 1e3:.1f} Mcoords/s, {steps / nc:.2f} steps/coord, "
          f"{gbs:.0f} GB/s algorithmic", flush=True)
