#!/bin/bash
# Chain timing experiments on the whole 'large' set (PROF=1 build paths): GB_CHAIN_EXP bits
# 1 producer skips the pair geometry, 2 consumer only drains the slots (outputs are garbage).
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
for e in ${EXPS:-0 1 2}; do
GB_CHAIN_PROF=1 GB_CHAIN_EXP=$e timeout -k 10 120 python - <<'PY' 2>&1 | grep -v "^\[chain prof\]" | head -3
import sys, os; sys.path.insert(0, '.')
from genomicsbench_palisade_amd import chain, gen, set_device
set_device(0)
calls = gen.chain_dataset("large", seed=5)
b = chain.ChainBatch(calls)
ms = []
for _ in range(3):
    b.run(); b.sync(); ms.append(b.timing())
print("exp", os.environ["GB_CHAIN_EXP"], min(ms), "ms")
PY
done
