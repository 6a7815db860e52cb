"""bsw lane-kernel utilisation probe (GB_BSW_PROF=1): per NCH variant, lane-row and column use."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genomicsbench_palisade_amd import bsw, gen, set_device
set_device(0)
p = gen.bsw_dataset(2_000_000, seed=11, threads=16)
b = bsw.BswBatch(p)
for _ in range(2):
    b.run(); b.sync()
    print("kernel ms", b.timing(), flush=True)
