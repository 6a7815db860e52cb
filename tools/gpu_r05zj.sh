#!/bin/bash
# round-5 GPU call zj: fmi GPU tests with the 5-entry head default (+ the head-size test), LDS-poison fmi
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zj}
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fmi_gpu.py tests/test_lds_poison.py \
  tests/test_fmi_large.py -m gpu > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
