"""chain_rows A/B probe: the 'large' set, the 'small' set and shard 0 of 8 of 'large', each with
GB_CHAIN_ROWS=0 (chain_kernel for every block) and 1 (chain_rows for sorted calls): ms per step (batch
events, best of 10 after 3 warm-ups), Manchors/s, and whether the two agree bit for bit on every
output. GB_CHAIN_SPLIT settings to try with rows on: CHAIN_SPLITS (';'-separated)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import chain, gen, set_device, shard  # noqa: E402

set_device(0)
large = gen.chain_dataset("large", seed=5)
lens = large.offsets[1:] - large.offsets[:-1]
c = int(np.argmax(lens))
o0, o1 = large.offsets[c], large.offsets[c + 1]
longest = gen.ChainCalls(np.array([0, o1 - o0]), large.x[o0:o1], large.y[o0:o1], large.avg_qspan[c:c + 1],
                         large.params4[c:c + 1])
sets = [("longest", longest), ("large", large), ("small", gen.chain_dataset("small", seed=5)),
        ("large 1/8", shard.shard_calls(large, 0, 8)[0])]
only = os.environ.get("CHAIN_SETS")
if only:
    sets = [s for s in sets if s[0] in only.split(",")]


def run(calls, rows, split=None):
    os.environ["GB_CHAIN_ROWS"] = rows
    if split is None:
        os.environ.pop("GB_CHAIN_SPLIT", None)
    else:
        os.environ["GB_CHAIN_SPLIT"] = split
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
    global last_stats
    last_stats = b.split_stats()
    b.close()
    return min(ks), res


last_stats = None


for name, calls in sets:
    sp = "0" if name == "longest" else None  # the longest call whole: per-anchor latency of one wave
    t0, r0 = run(calls, "0", sp)
    t1, r1 = run(calls, "1", sp)
    same = all(np.array_equal(a, b) for a, b in zip(r0[:4], r1[:4])) and r0[4] == r1[4]
    print(f"{name:10s} {calls.nanchors:9d} anchors: chain_kernel {t0:7.3f} ms ({calls.nanchors / t0 / 1e3:7.1f} "
          f"Manchors/s), chain_rows {t1:7.3f} ms ({calls.nanchors / t1 / 1e3:7.1f} Manchors/s), same={same}",
          flush=True)
    for s in [x for x in os.environ.get("CHAIN_SPLITS", "").split(";") if x]:
        ts, rs = run(calls, "1", s)
        ok = all(np.array_equal(a, b) for a, b in zip(r0[:4], rs[:4])) and r0[4] == rs[4]
        print(f"   rows, split {s:10s}: {ts:7.3f} ms ({calls.nanchors / ts / 1e3:7.1f} Manchors/s) same={ok} "
              f"(split calls, rounds, fix-ups {last_stats})", flush=True)
