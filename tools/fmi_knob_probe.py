"""fmi knob sweep: the 'large' read set (10 M reads over the 512 Mbp index) and its 1/8 shard searched
under each environment setting in FMI_CONFIGS (';'-separated, each VAR=VALUE joined by '+', '' =
defaults), e.g. FMI_CONFIGS=";GB_FMI_WAVES_PER_CU=12;GB_FMI_TOP=4+GB_FMI_WAVES_PER_CU=16". The knobs
apply to a read set made after they are set, so one process times them all on one index. Prints the best of
4 searches (wall and kernel-event ms) and whether the SMEM totals equal the default's."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import genomicsbench_palisade_amd as g  # noqa: E402
if os.environ.get("FMI_LIB"):  # another build of libgb.so, to time two builds on one box
    g.LIBGB = os.path.abspath(os.environ["FMI_LIB"])
from genomicsbench_palisade_amd import fmi, gen, set_device, shard  # noqa: E402

KNOBS = ("GB_FMI_WAVES_PER_CU", "GB_FMI_TOP", "GB_FMI_HEAVY", "GB_FMI_QLDS", "GB_FMI_PREFETCH", "GB_FMI_SPLIT", "GB_FMI_Q2")
set_device(0)
nreads = int(os.environ.get("FMI_PROBE_READS", "10000000"))
ref = gen.fmi_reference(512_000_000, seed=7)
idx = fmi.Index.build(ref)
codes, lens = gen.fmi_reads(ref, nreads, read_len=151, seed=8)
lo, hi = shard.read_range(nreads, 0, 8)
configs = os.environ.get("FMI_CONFIGS", "").split(";")
for name, (a, b) in (("full", (0, nreads)), ("shard0/8", (lo, hi))):
    base = None
    for cfg in configs:
        for k in KNOBS:
            os.environ.pop(k, None)
        for kv in [c for c in cfg.split("+") if c]:
            k, v = kv.split("=", 1)
            os.environ[k] = v
        rs = fmi.Reads(idx, codes[a:b], lens[a:b])  # the grid size is fixed when the read set is made
        rs.search(19)
        rs.sync()
        best, kbest = 1e9, 1e9
        for _ in range(4):
            t0 = time.perf_counter()
            rs.search(19)
            rs.sync()
            best = min(best, time.perf_counter() - t0)
            kbest = min(kbest, rs.timing()[0])
        _, tot, _, _ = rs.results(batch_size=512, want_smems=False)
        base = tot if base is None else base
        print(f"{os.path.basename(g.LIBGB)} {name:8s} [{cfg or 'default':45s}] wall {best * 1e3:8.2f} ms, search {kbest:8.2f} ms "
              f"({(b - a) / best / 1e6:6.2f} Mreads/s) smems {tot} same={tot == base}", flush=True)
        rs.close()
idx.close()
