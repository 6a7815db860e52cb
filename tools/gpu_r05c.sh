#!/bin/bash
# round-5 GPU call c: 'small'-set floors -- bsw tail fraction sweep and fmi heavy-read budget sweep on
# the small sets and their 1/8 shards
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05c}
BSW_PAIRS=100000 BSW_REBUILD=1 BSW_CONFIGS=";GB_BSW_TAIL=0;GB_BSW_TAIL=0.3;GB_BSW_TAIL=0.5;GB_BSW_TAIL=0.7;GB_BSW_TAIL=0.9;GB_BSW_TAIL=1" \
  timeout -k 10 300 python -u tools/bsw_knob_probe.py > gpurun_out/bsw_tail_${T}.log 2>&1 || { tail -20 gpurun_out/bsw_tail_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bsw_tail_${T}.log
FMI_PROBE_READS=1000000 FMI_CONFIGS=";GB_FMI_HEAVY=1000;GB_FMI_HEAVY=500;GB_FMI_HEAVY=250;GB_FMI_HEAVY=120;GB_FMI_WAVES_PER_CU=8;GB_FMI_WAVES_PER_CU=24" \
  timeout -k 10 400 python -u tools/fmi_knob_probe.py > gpurun_out/fmi_heavy_${T}.log 2>&1 || { tail -20 gpurun_out/fmi_heavy_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/fmi_heavy_${T}.log
