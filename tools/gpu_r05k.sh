#!/bin/bash
# round-5 GPU call k: phmm (pinned staging) + chain (row target) parity, bin/phmm host profile, chain
# sets under the new defaults
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05k}
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_phmm_gpu.py tests/test_chain.py \
  tests/test_edges.py -m gpu > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
PHMM_CLI_CONFIGS=";GB_PHMM_HOSTPROF=1;GB_PHMM_PIPE=2" timeout -k 10 300 python -u tools/phmm_cli_probe.py \
  > gpurun_out/phmm_cli_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_cli_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_cli_${T}.log | cut -c1-1500
timeout -k 10 200 python -u tools/phmm_cold_probe.py > gpurun_out/phmm_cold_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_cold_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_cold_${T}.log
CHAIN_CONFIGS=";GB_CHAIN_TARGET=0" timeout -k 10 300 python -u tools/chain_knob_probe.py > gpurun_out/chain_target_${T}.log 2>&1 \
  || { tail -20 gpurun_out/chain_target_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/chain_target_${T}.log
