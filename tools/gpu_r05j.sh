#!/bin/bash
# round-5 GPU call j: phmm pipelined fetch order + bin/phmm host profile; chain per-call segment
# lengths under a row target (GB_CHAIN_TARGET) on the large / small sets and their 1/8 shards
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05j}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_phmm_gpu.py -m gpu \
  > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
PHMM_CLI_CONFIGS=";GB_PHMM_HOSTPROF=1;GB_PHMM_PIPE=2" timeout -k 10 300 python -u tools/phmm_cli_probe.py \
  > gpurun_out/phmm_cli_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_cli_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_cli_${T}.log | cut -c1-1500
timeout -k 10 200 python -u tools/phmm_cold_probe.py > gpurun_out/phmm_cold_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_cold_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_cold_${T}.log
CHAIN_CONFIGS=";GB_CHAIN_TARGET=900;GB_CHAIN_TARGET=800;GB_CHAIN_TARGET=700;GB_CHAIN_TARGET=600" timeout -k 10 500 python -u tools/chain_knob_probe.py \
  > gpurun_out/chain_target_${T}.log 2>&1 || { tail -20 gpurun_out/chain_target_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/chain_target_${T}.log
