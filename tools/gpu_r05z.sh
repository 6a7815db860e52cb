#!/bin/bash
# round-5 GPU call z: fmi hand-over budget / occupancy on the 'large' set and its 1/8 shard
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05z}
FMI_CONFIGS="${FMI_CONFIGS:-;GB_FMI_HEAVY=1600;GB_FMI_HEAVY=1800;GB_FMI_HEAVY=2500;GB_FMI_WAVES_PER_CU=18;GB_FMI_WAVES_PER_CU=14}" \
  timeout -k 10 600 python -u tools/fmi_knob_probe.py > gpurun_out/fmi_knobs_${T}.log 2>&1 || { tail -20 gpurun_out/fmi_knobs_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/fmi_knobs_${T}.log
