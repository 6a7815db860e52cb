#!/bin/bash
# round-5 GPU call zz9: chain tests and the four chain sets after the shorter segment floor and
# warm-up under the row target
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zz9}
timeout -k 10 400 python -u -m pytest tests/test_chain.py tests/test_lds_poison.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/chain_tests_${T}.log 2>&1 || { tail -30 gpurun_out/chain_tests_${T}.log; exit 1; }
tail -2 gpurun_out/chain_tests_${T}.log
CHAIN_SETS=s_shard0/8,small,shard0/8,large CHAIN_CONFIGS=";GB_CHAIN_SEGMIN=128+GB_CHAIN_SPLIT=-1,32" \
  timeout -k 10 400 python -u tools/chain_knob_probe.py > gpurun_out/chain_knobs_${T}.log 2>&1 || { tail -20 gpurun_out/chain_knobs_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/chain_knobs_${T}.log
