"""bsw knob sweep: the 'large' pair set (10.6 M pairs) and its 1/8 shard run under each environment
setting in BSW_CONFIGS (';'-separated, each VAR=VALUE joined by '+', '' = defaults), e.g.
    BSW_CONFIGS=";GB_BSW_SMALL=0" python tools/bsw_knob_probe.py
(round 4 timed the lane-refill experiment's GB_BSW_REFILL with it, profiles/r04i_bsw_refill_ab.log)
The knobs are read at every run, so one batch serves all settings. Per setting: best-of-5 batch-event
ms per step, GCUPS, and whether out6 and the cell counts equal the first setting's (bit for bit)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import genomicsbench_palisade_amd as g  # noqa: E402
if os.environ.get("BSW_LIB"):  # another build of libgb.so, to time two builds on one box
    g.LIBGB = os.path.abspath(os.environ["BSW_LIB"])
from genomicsbench_palisade_amd import bsw, gen, set_device, shard  # noqa: E402

KNOBS = ("GB_BSW_REFILL", "GB_BSW_PROF", "GB_BSW_SMALL", "GB_BSW_H0STEP", "GB_BSW_QSHIFT", "GB_BSW_KEYORD",
         "GB_BSW_TAIL")
set_device(0)
# BSW_PAIRS: the set size (default the 'large' set; gen.BSW_SMALL_PAIRS for 'small')
pairs = gen.bsw_dataset(int(os.environ["BSW_PAIRS"]), seed=11, threads=16) if os.environ.get("BSW_PAIRS") \
    else gen.bsw_dataset(seed=11, threads=16)
sets = [("large", pairs)]
if os.environ.get("BSW_SHARD", "1") == "1":
    sets.append(("shard0/8", shard.shard_pairs(pairs, 0, 8)[0]))
configs = os.environ.get("BSW_CONFIGS", "").split(";")
for name, ps in sets:
    if ps is None:
        continue
    b = bsw.BswBatch(ps)
    base = None
    for cfg in configs:
        for k in KNOBS:
            os.environ.pop(k, None)
        for kv in [c for c in cfg.split("+") if c]:
            k, v = kv.split("=", 1)
            os.environ[k] = v
        if os.environ.get("BSW_REBUILD") == "1":  # knobs read when a batch is made (GB_BSW_KEY)
            b.close()
            b = bsw.BswBatch(ps)
        b.run()
        b.sync()
        best = 1e9
        for _ in range(5):
            b.run()
            b.sync()
            best = min(best, b.timing())
        out6, cells, tot = b.results()
        if base is None:
            base = (out6, cells)
        same = np.array_equal(out6, base[0]) and np.array_equal(cells, base[1])
        print(f"{os.path.basename(g.LIBGB)} {name:8s} [{cfg or 'default':32s}] {best:8.3f} ms  {tot / best / 1e6:8.1f} GCUPS  same={same}", flush=True)
    b.close()
