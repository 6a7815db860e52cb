#!/bin/bash
# round-5 GPU call zh: fmi 6-entry prev head: parity under GB_FMI_TOP=6, timing against 4 / 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zh}
GB_FMI_TOP=6 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fmi_gpu.py -m gpu \
  > gpurun_out/pytest_${T}.log 2>&1 || { tail -40 gpurun_out/pytest_${T}.log; exit 1; }
tail -1 gpurun_out/pytest_${T}.log
FMI_CONFIGS=";GB_FMI_TOP=6;GB_FMI_TOP=6+GB_FMI_WAVES_PER_CU=13;GB_FMI_TOP=8" timeout -k 10 600 python -u tools/fmi_knob_probe.py \
  > gpurun_out/fmi_top6_${T}.log 2>&1 || { tail -20 gpurun_out/fmi_top6_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/fmi_top6_${T}.log
