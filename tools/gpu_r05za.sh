#!/bin/bash
# round-5 GPU call za: bsw tail rule on the 'large' set and its 1/8 shard
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05za}
BSW_CONFIGS="${BSW_CONFIGS:-;GB_BSW_TAILMAX=100+GB_BSW_TAIL=0.01;GB_BSW_TAILMAX=100+GB_BSW_TAIL=0.02;GB_BSW_TAILMAX=100+GB_BSW_TAIL=0.05;GB_BSW_TAILMAX=100+GB_BSW_TAIL=0.1}" \
  timeout -k 10 500 python -u tools/bsw_knob_probe.py > gpurun_out/bsw_tail_${T}.log 2>&1 || { tail -20 gpurun_out/bsw_tail_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bsw_tail_${T}.log
