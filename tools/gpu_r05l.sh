#!/bin/bash
# round-5 GPU call l: phmm concurrent chunk fills + init preallocation: parity, bin/phmm, cold calls
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05l}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_phmm_gpu.py tests/test_edges.py \
  -m gpu > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
PHMM_CLI_CONFIGS="${CLI_CONFIGS:-;GB_PHMM_HOSTPROF=1;GB_PHMM_FILL_THREADS=6;GB_PHMM_FILL_THREADS=2;GB_PHMM_PIPE=6}" \
  timeout -k 10 300 python -u tools/phmm_cli_probe.py > gpurun_out/phmm_cli_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_cli_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_cli_${T}.log | cut -c1-2500
timeout -k 10 200 python -u tools/phmm_cold_probe.py > gpurun_out/phmm_cold_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_cold_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_cold_${T}.log
