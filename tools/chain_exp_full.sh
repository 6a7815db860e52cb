#!/bin/bash
# Chain timing experiments (PROF=1 build paths) on the calls of the 'large' set short enough to run
# whole (< 8192 anchors, no speculative segments: the experiments' outputs are garbage):
# GB_CHAIN_EXP bits 1 producer skips the pair geometry, 2 consumer only drains the slots.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
for e in ${EXPS:-0 1 2}; do
GB_CHAIN_SPLIT=0 GB_CHAIN_PROF=1 GB_CHAIN_EXP=$e timeout -k 10 120 python - <<'PY' 2>&1 | grep -v "^\[chain prof\]" | head -3
import sys, os; sys.path.insert(0, '.')
from genomicsbench_palisade_amd import chain, gen, set_device
set_device(0)
import numpy as np
calls = gen.chain_dataset("large", seed=5)
lens = calls.offsets[1:] - calls.offsets[:-1]
idx = np.nonzero(lens < 8192)[0]
sel = np.concatenate([np.arange(calls.offsets[c], calls.offsets[c + 1]) for c in idx])
offs = np.zeros(len(idx) + 1, np.int64); offs[1:] = np.cumsum(lens[idx])
sub = gen.ChainCalls(offs, calls.x[sel], calls.y[sel], calls.avg_qspan[idx], calls.params4[idx])
print("calls", sub.ncalls, "anchors", sub.nanchors)
b = chain.ChainBatch(sub)
ms = []
for _ in range(3):
    b.run(); b.sync(); ms.append(b.timing())
print("exp", os.environ["GB_CHAIN_EXP"], min(ms), "ms")
PY
done
