#!/bin/bash
# round-5 GPU call f: parity of chain (one clear kernel per step) and phmm (init warm-up, f64 units),
# chain shard timings, bin/phmm end to end
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05f}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_chain.py tests/test_edges.py \
  tests/test_phmm_gpu.py tests/test_lds_poison.py -m gpu > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
for kind in large small; do
  CHAIN_KIND=$kind timeout -k 10 300 python -u tools/chain_shard_probe.py > gpurun_out/chain_shard_${kind}_${T}.log 2>&1 \
    || { tail -20 gpurun_out/chain_shard_${kind}_${T}.log; exit 1; }
  CHAIN_KIND=$kind CHAIN_OF=1 timeout -k 10 300 python -u tools/chain_shard_probe.py >> gpurun_out/chain_shard_${kind}_${T}.log 2>&1 \
    || { tail -20 gpurun_out/chain_shard_${kind}_${T}.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/chain_shard_${kind}_${T}.log
done
PHMM_CLI_CONFIGS=";GB_PHMM_PIPE=2;GB_PHMM_HOSTPROF=1" timeout -k 10 300 python -u tools/phmm_cli_probe.py \
  > gpurun_out/phmm_cli_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_cli_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_cli_${T}.log | cut -c1-900
