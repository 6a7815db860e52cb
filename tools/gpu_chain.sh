#!/bin/bash
# Chain development run on the GPU box: light profile stamps (GB_CHAIN_PROF=1: grid span, start/end of
# the longest call) for the longest call alone and for the whole 'large' set, the chain_dp and
# backtrack GPU parity tests, and tools/chain_probe.py (whole set / longest call / the rest).
#   gpurun --timeout 900 -- 'bash tools/gpu_chain.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
GB_CHAIN_PROF=${PROFLEVEL:-1} timeout -k 10 300 python - > gpurun_out/chain_prof.log 2>&1 <<'PY' || { tail gpurun_out/chain_prof.log; exit 1; }
import sys; sys.path.insert(0, '.'); sys.path.insert(0, 'tools')
import numpy as np
from genomicsbench_palisade_amd import chain, gen, set_device
set_device(0)
calls = gen.chain_dataset("large", seed=5)
lens = calls.offsets[1:] - calls.offsets[:-1]
c = int(np.argmax(lens))
o0, o1 = calls.offsets[c], calls.offsets[c + 1]
sub = gen.ChainCalls(np.array([0, o1 - o0]), calls.x[o0:o1], calls.y[o0:o1], calls.avg_qspan[c:c+1], calls.params4[c:c+1])
for name, cc in [("longest", sub), ("all", calls)]:
    b = chain.ChainBatch(cc)
    for _ in range(2):
        b.run(); b.sync()
    print(name, b.timing(), "ms", flush=True)
PY
cat gpurun_out/chain_prof.log
timeout -k 10 400 python -u -m pytest tests/test_chain.py tests/test_chain_bt.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/chain_test.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/chain_test.log; exit 1; }
tail -1 gpurun_out/chain_test.log
timeout -k 10 300 python tools/chain_probe.py > gpurun_out/chain_probe.log 2>&1 || { tail gpurun_out/chain_probe.log; exit 1; }
cat gpurun_out/chain_probe.log
