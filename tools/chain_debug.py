"""chain bisection probe: one generated set (test_gpu_vs_oracle's first case by default) against the
oracle under each setting of CHAIN_CONFIGS (as tools/chain_knob_probe.py) and each library of
CHAIN_LIBS (':'-separated libgb.so builds, in separate processes): per output, the number of anchors
that differ and the first one."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

if len(sys.argv) == 1:
    for lib in os.environ.get("CHAIN_LIBS", os.path.join(ROOT, "genomicsbench_palisade_amd/lib/libgb.so")).split(":"):
        r = subprocess.run([sys.executable, __file__, lib], timeout=300)
        if r.returncode:
            sys.exit(r.returncode)
    sys.exit(0)

import genomicsbench_palisade_amd as g  # noqa: E402
g.LIBGB = os.path.abspath(sys.argv[1])
import oracle_lib  # noqa: E402
from genomicsbench_palisade_amd import chain, gen, set_device  # noqa: E402

set_device(0)
seed, ncalls, median, maxn = (int(v) for v in os.environ.get("CHAIN_SET", "1,300,1500,87271").split(","))
calls = gen.chain_dataset("small", num_calls=ncalls, seed=seed, median_n=median, max_n=maxn)
exp = oracle_lib.chain_oracle(calls, 8)
KNOBS = ("GB_CHAIN_SPLIT", "GB_CHAIN_ROWS", "GB_CHAIN_VLANES", "GB_CHAIN_PRIO")
for cfg in os.environ.get("CHAIN_CONFIGS", "").split(";"):
    for k in KNOBS:
        os.environ.pop(k, None)
    for kv in [c for c in cfg.split("+") if c]:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    b = chain.ChainBatch(calls)
    b.run()
    got = b.results()
    st = b.split_stats()
    b.close()
    out = []
    for name, gv, ev in zip(("score", "parent", "target", "peak"), got[:4], exp[:4]):
        bad = np.nonzero(gv != ev)[0]
        out.append(f"{name} {len(bad)}" + (f" (first {bad[0]}: {gv[bad[0]]} vs {ev[bad[0]]})" if len(bad) else ""))
    out.append(f"visited {got[4]} vs {exp[4]}")
    print(f"[{os.path.basename(g.LIBGB)}] [{cfg or 'default'}] split {st}: " + ", ".join(out), flush=True)
