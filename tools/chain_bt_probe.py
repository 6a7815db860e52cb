"""chain backtrack probe: the 'large' set's chain_dp outputs, backtrack (min_cnt 3, min_sc 40) timed by
the batch events (best of 10 after 3 warm-ups), and the chains checked against the first run's."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from genomicsbench_palisade_amd import chain, gen, set_device  # noqa: E402

set_device(0)
calls = gen.chain_dataset(os.environ.get("BT_SET", "large"), seed=5)
b = chain.ChainBatch(calls)
b.run()
b.sync()
ts = []
ref = None
for k in range(13):
    b.backtrack(3, 40)
    got = b.chains()
    if ref is None:
        ref = got
    else:
        assert all(np.array_equal(np.asarray(a), np.asarray(c)) for a, c in zip(ref, got)), "backtrack differs between runs"
    if k >= 3:
        ts.append(b.backtrack_timing())
print(f"backtrack {calls.nanchors} anchors: {min(ts):.3f} ms ({calls.nanchors / min(ts) / 1e3:.1f} Manchors/s)")
