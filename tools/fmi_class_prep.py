"""Inputs for the FMI_search class drop-in probe: the bench's fmi 'large' reference (512 Mbp,
seed 7) as <dir>/ref.bwt.2bit.64 and the first N reads of its read set (seed 8) as <dir>/reads.bin,
the layout tests/cpp/fmi_class_driver.cpp reads.
    python tools/fmi_class_prep.py <dir> [reads] [mbp]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import fmi, gen, set_device  # noqa: E402

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
mbp = float(sys.argv[3]) if len(sys.argv) > 3 else 512
os.makedirs(d, exist_ok=True)
set_device(0)
ref = gen.fmi_reference(int(mbp * 1e6), seed=7)
codes, lens = gen.fmi_reads(ref, n, read_len=151, seed=8)
fmi.Index.build(ref, out_path=os.path.join(d, "ref.bwt.2bit.64")).close()
with open(os.path.join(d, "reads.bin"), "wb") as f:
    f.write(np.array([n, codes.shape[1]], np.int32).tobytes() + lens.astype(np.int32).tobytes()
            + np.ascontiguousarray(codes).tobytes())
print(f"prepared {n} reads over {mbp} Mbp in {d}", flush=True)
