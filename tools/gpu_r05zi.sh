#!/bin/bash
# round-5 GPU call zi: fmi prev-head sizes 5 / 6 / 7 (and occupancy around 6)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zi}
FMI_CONFIGS="${CFG:-GB_FMI_TOP=6;GB_FMI_TOP=5;GB_FMI_TOP=7;GB_FMI_TOP=6+GB_FMI_WAVES_PER_CU=15;;GB_FMI_TOP=6}" timeout -k 10 600 python -u tools/fmi_knob_probe.py \
  > gpurun_out/fmi_top_${T}.log 2>&1 || { tail -20 gpurun_out/fmi_top_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/fmi_top_${T}.log
