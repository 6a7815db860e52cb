#!/bin/bash
# round-5 GPU call d: phmm + bsw parity after the pipeline / routing changes, bin/phmm end to end
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05d}
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_phmm_gpu.py tests/test_bsw.py -m gpu \
  > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
PHMM_CLI_CONFIGS=";GB_PHMM_PIPE=1;GB_PHMM_PIPE=2;GB_PHMM_PIPE=3;GB_PHMM_HOSTPROF=1" timeout -k 10 300 python -u tools/phmm_cli_probe.py \
  > gpurun_out/phmm_cli_${T}.log 2>&1 || { tail -20 gpurun_out/phmm_cli_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phmm_cli_${T}.log | cut -c1-900
