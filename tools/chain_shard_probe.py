"""chain strong-scaling shard probe: rank CHAIN_RANK (default 0) of CHAIN_OF (default 8) of the 'large'
set, timed per GB_CHAIN_SPLIT setting in CHAIN_SPLITS (';'-separated, 'default' = the adaptive
choice): wall ms per step (sync'd), the batch's own event time, split statistics."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import chain, gen, set_device, shard  # noqa: E402

set_device(0)
full = gen.chain_dataset(os.environ.get("CHAIN_KIND", "large"), seed=5)  # CHAIN_KIND=small: the 'small' set
of, r = int(os.environ.get("CHAIN_OF", "8")), int(os.environ.get("CHAIN_RANK", "0"))
calls, (lo, hi) = shard.shard_calls(full, r, of) if of > 1 else (full, (0, full.ncalls))
print(f"shard {r}/{of}: calls {lo}..{hi}, {calls.nanchors} anchors", flush=True)
for s in os.environ.get("CHAIN_SPLITS", "default").split(";"):
    if s == "default":
        os.environ.pop("GB_CHAIN_SPLIT", None)
    else:
        os.environ["GB_CHAIN_SPLIT"] = s
    b = chain.ChainBatch(calls)
    for _ in range(3):
        b.run()
        b.sync()
    steps = 10
    t0 = time.perf_counter()
    ks = []
    for _ in range(steps):
        b.run()
        b.sync()
        ks.append(b.timing())
    wall = (time.perf_counter() - t0) / steps * 1e3
    st = b.split_stats()
    b.close()
    print(f"split {s:10s}: wall {wall:7.3f} ms/step ({calls.nanchors / wall / 1e3:8.1f} Manchors/s), events "
          f"{min(ks):7.3f} ms; split calls {st[0]}, rounds {st[1]}, fix-ups {st[2]}", flush=True)
