"""fmi search probe: synthetic index (FMI_PROBE_MBP, default 512 Mbp) and FMI_PROBE_READS reads
(default 4M), timed search for each GB_FMI_FLAGS value in FMI_PROBE_FLAGS (default "0")."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genomicsbench_palisade_amd import fmi, gen, set_device
set_device(0)
mbp = float(os.environ.get("FMI_PROBE_MBP", "512"))
nreads = int(os.environ.get("FMI_PROBE_READS", "4000000"))
ref = gen.fmi_reference(int(mbp * 1e6), seed=7)
idx = fmi.Index.build(ref)
codes, lens = gen.fmi_reads(ref, nreads, read_len=151, seed=8)
rs = fmi.Reads(idx, codes, lens)
for rep in range(2):
    for fl in os.environ.get("FMI_PROBE_FLAGS", "0").split(","):
        os.environ["GB_FMI_FLAGS"] = fl
        rs.search(19)
        rs.sync()
        a, b, calls = rs.timing()
        extra = ""
        if int(fl) & 4:
            import ctypes
            import numpy as np
            from genomicsbench_palisade_amd import lib
            pr = np.zeros(8, np.uint64)
            lib().gb_fmi_debug_prof(ctypes.c_void_p(pr.ctypes.data), 1)
            tot = float(pr[:3].sum())
            extra = (f" | per wave-trip: state {pr[0] / pr[3]:.0f} gather {pr[1] / pr[3]:.0f} consume {pr[2] / pr[3]:.0f} clk"
                     f" ({pr[0] / tot:.2f}/{pr[1] / tot:.2f}/{pr[2] / tot:.2f}), {int(pr[3])} wave-trips;"
                     f" lane state iters/lane-trip {pr[4] / pr[3] / 64:.2f}; new-read trips {pr[5] / pr[3]:.3f}"
                     f" with state {pr[6] / max(pr[5], 1):.0f} clk (share of state time {pr[6] / pr[0]:.2f})")
        print(f"flags {fl}: search {a:.2f} ms total {b:.2f} ms, {calls / nreads:.1f} ext/read, {nreads / a / 1e3:.2f} Mreads/s{extra}", flush=True)
