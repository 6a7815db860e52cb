"""chain knob sweep: the 'large' set and its shard 0 of 8 under each environment setting in
CHAIN_CONFIGS (';'-separated, each a ','-free list of VAR=VALUE joined by '+', '' = defaults), e.g.
    CHAIN_CONFIGS=";GB_CHAIN_SPLIT=512,128,0,512;GB_CHAIN_ROWS_MAXN=1024" python tools/chain_knob_probe.py
Per set and setting: batch-event ms per step (best of 10 after 3 warm-ups), Manchors/s, split
statistics and whether every output equals the default setting's (bit for bit)."""
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import genomicsbench_palisade_amd as g  # noqa: E402
if os.environ.get("CHAIN_LIB"):  # another build of libgb.so, to time two builds on one box
    g.LIBGB = os.path.abspath(os.environ["CHAIN_LIB"])
from genomicsbench_palisade_amd import chain, gen, set_device, shard  # noqa: E402

set_device(0)
large = gen.chain_dataset("large", seed=5)
small = gen.chain_dataset("small", seed=5)
sets = [("shard0/8", shard.shard_calls(large, 0, 8)[0]), ("large", large),
        ("s_shard0/8", shard.shard_calls(small, 0, 8)[0]), ("small", small)]
if os.environ.get("CHAIN_SETS"):
    sets = [s for s in sets if s[0] in os.environ["CHAIN_SETS"].split(",")]
configs = os.environ.get("CHAIN_CONFIGS", "").split(";")
KNOBS = ("GB_CHAIN_SPLIT", "GB_CHAIN_ROWS", "GB_CHAIN_ROWS_MAXN", "GB_CHAIN_VLANES", "GB_CHAIN_PRIO", "GB_CHAIN_SPREAD",
         "GB_CHAIN_EXP", "GB_CHAIN_TARGET", "GB_CHAIN_SEGMIN")


def parse_cfg(cfg):
    """'VAR=VALUE+VAR=VALUE' -> ['VAR=VALUE', ...]; a '+' only separates settings when a knob name
    follows it, and anything else is refused with the offending setting named (round 4's probe died
    with a bare ValueError on a malformed setting, profiles/r04zj_chain_warm_ab.log)."""
    parts = [c for c in re.split(r"\+(?=GB_)", cfg) if c]
    for kv in parts:
        if "=" not in kv or kv.split("=", 1)[0] not in KNOBS:
            raise SystemExit(f"chain_knob_probe: bad setting {kv!r} in CHAIN_CONFIGS entry {cfg!r} "
                             f"(want VAR=VALUE with VAR one of {', '.join(KNOBS)})")
    return parts


def run(calls, cfg):
    for k in KNOBS:
        os.environ.pop(k, None)
    for kv in parse_cfg(cfg):
        k, v = kv.split("=", 1)
        os.environ[k] = v
    b = chain.ChainBatch(calls)
    for _ in range(3):
        b.run()
        b.sync()
    ks = []
    for _ in range(10):
        b.run()
        b.sync()
        ks.append(b.timing())
    res = b.results()
    st = b.split_stats()
    b.close()
    return min(ks), res, st


for name, calls in sets:
    base = None
    for cfg in configs:
        t, r, st = run(calls, cfg)
        if base is None:
            base = r
        same = all(np.array_equal(a, b) for a, b in zip(base[:4], r[:4])) and base[4] == r[4]
        print(f"{os.path.basename(g.LIBGB)} {name:9s} [{cfg or 'default':40s}] {t:7.3f} ms ({calls.nanchors / t / 1e3:7.1f} Manchors/s) "
              f"split calls/rounds/fix-ups {st} same={same}", flush=True)
