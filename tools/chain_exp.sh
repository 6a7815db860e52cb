cd ${GRAFT_REPO_ROOT}
for e in ${EXPS:-0 1 2 3}; do
GB_CHAIN_PROF=1 GB_CHAIN_EXP=$e timeout -k 10 120 python - <<'PY' 2>&1 | grep -v "^\[chain prof\] longest" | head -3
import sys, os; sys.path.insert(0, '.')
import numpy as np
from genomicsbench_palisade_amd import chain, gen, set_device
set_device(0)
calls = gen.chain_dataset("large", seed=5)
lens = calls.offsets[1:] - calls.offsets[:-1]
c = int(np.argmax(lens))
sub = calls.slice(c, c + 1)
b = chain.ChainBatch(sub)
b.run(); b.sync()
b.run(); b.sync()
print("exp", os.environ["GB_CHAIN_EXP"], b.timing(), "ms")
PY
done
