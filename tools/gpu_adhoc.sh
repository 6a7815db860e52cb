#!/bin/bash
# scratch GPU session (edited per experiment; the checkpoints use tools/gpu_checkpoint.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_checkpoint.sh r04f tests smoke bench prof || exit 1
FMI_CONFIGS=";GB_FMI_TOP=0+GB_FMI_WAVES_PER_CU=16;GB_FMI_TOP=4+GB_FMI_WAVES_PER_CU=14;GB_FMI_TOP=8+GB_FMI_WAVES_PER_CU=11" \
  timeout -k 10 300 python3 tools/fmi_knob_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/fmi_knobs_r04f.log || exit 1
