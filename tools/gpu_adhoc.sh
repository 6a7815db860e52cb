#!/bin/bash
# scratch GPU session (edited per experiment; the checkpoints use tools/gpu_checkpoint.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04o
FMI_CONFIGS=";GB_FMI_HEAVY=700;GB_FMI_HEAVY=1000;GB_FMI_HEAVY=1400;GB_FMI_HEAVY=3000;GB_FMI_WAVES_PER_CU=15;GB_FMI_WAVES_PER_CU=17" \
  timeout -k 10 400 python3 tools/fmi_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/fmi_knobs_$T.log || exit 1
