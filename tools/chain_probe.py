"""Chain kernel timing probe: whole 'large' set vs its longest call alone vs the rest."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import genomicsbench_palisade_amd as gbp
if os.environ.get("GB_LIBGB"):  # A/B a differently built libgb.so (development aid)
    gbp.LIBGB = os.path.abspath(os.environ["GB_LIBGB"])
from genomicsbench_palisade_amd import chain, gen, set_device

set_device(0)
calls = gen.chain_dataset("large", seed=5)


def sub(idx):
    idx = np.sort(np.asarray(idx))
    lens = calls.offsets[idx + 1] - calls.offsets[idx]
    offs = np.zeros(len(idx) + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    sel = np.concatenate([np.arange(calls.offsets[c], calls.offsets[c + 1]) for c in idx])
    return gen.ChainCalls(offs, calls.x[sel], calls.y[sel], calls.avg_qspan[idx], calls.params4[idx])


def t(c, reps=3):
    b = chain.ChainBatch(c)
    ms = []
    for _ in range(reps):
        b.run(); b.sync(); ms.append(b.timing())
    v = b.results()[4]
    st = b.split_stats()
    b.close()
    return min(ms), v, st


lens = calls.offsets[1:] - calls.offsets[:-1]
order = np.argsort(-lens)
for name, idx in [("all", np.arange(calls.ncalls)), ("longest", order[:1]), ("top8", order[:8]),
                  ("rest", order[1:]), ("short_half", order[calls.ncalls // 2:])]:
    c = sub(idx)
    ms, v, st = t(c)
    print(f"{name:10s} calls {c.ncalls:6d} anchors {c.nanchors:9d} visited {v:11d} kernel {ms:8.2f} ms "
          f"-> {ms * 1e6 / max(lens[idx].max(), 1):.1f} ns per anchor of the longest call; split calls, rounds, "
          f"fix-ups {st}", flush=True)
