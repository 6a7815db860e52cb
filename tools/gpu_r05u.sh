#!/bin/bash
# round-5 GPU call u: phmm GPU tests (new pipelined cases)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05u}
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_phmm_gpu.py -m gpu \
  > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/pytest_${T}.log | tail -30
