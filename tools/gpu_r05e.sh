#!/bin/bash
# round-5 GPU call e: phmm parity (arena buffers, f64 work units), f64 work-unit split A/B on the
# 1/8 shard, bin/phmm end to end (threaded testcase construction)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05e}
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_phmm_gpu.py tests/test_edges.py -m gpu \
  > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
GB_PHMM_F64_PARTS=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_phmm_gpu.py -m gpu \
  -k "golden or random or stack_edges" > gpurun_out/pytest_${T}_parts.log 2>&1 || { tail -40 gpurun_out/pytest_${T}_parts.log; exit 1; }
tail -1 gpurun_out/pytest_${T}_parts.log
PHMM_ROWS="default;GB_PHMM_F64_PARTS=2;GB_PHMM_F64_PARTS=4;default" timeout -k 10 300 python -u tools/phmm_shard_probe.py \
  > gpurun_out/phmm_parts_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_parts_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_parts_${T}.log
PHMM_CLI_CONFIGS=";GB_PHMM_PIPE=1;GB_PHMM_PIPE=2;GB_PHMM_PIPE=3;GB_PHMM_HOSTPROF=1" timeout -k 10 300 python -u tools/phmm_cli_probe.py \
  > gpurun_out/phmm_cli_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_cli_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_cli_${T}.log | cut -c1-900
