#!/bin/bash
# round-5 GPU call r: bsw grouped vs whole-wave mode in one build (small set + shard)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05r}
BSW_PAIRS=100000 BSW_CONFIGS="${BSW_CONFIGS:-;GB_BSW_GROUP=0;GB_BSW_TAIL=0.1;GB_BSW_TAIL=0.1+GB_BSW_GROUP=0}" timeout -k 10 300 python -u tools/bsw_knob_probe.py \
  > gpurun_out/bsw_small_${T}.log 2>&1 || { tail -20 gpurun_out/bsw_small_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bsw_small_${T}.log
