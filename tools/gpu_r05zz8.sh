#!/bin/bash
# round-5 GPU call zz8: chain 'small' and its 1/8 shard under shorter segments / warm-ups below the
# row target (GB_CHAIN_SEGMIN, GB_CHAIN_SPLIT's warm-up)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zz8}
CHAIN_SETS=${SETS:-s_shard0/8,small} CHAIN_CONFIGS="${CFG:-;GB_CHAIN_SEGMIN=96;GB_CHAIN_SEGMIN=64;GB_CHAIN_SEGMIN=32;GB_CHAIN_SPLIT=-1,16;GB_CHAIN_SEGMIN=64+GB_CHAIN_SPLIT=-1,16;GB_CHAIN_SEGMIN=64+GB_CHAIN_TARGET=500}" \
  timeout -k 10 600 python -u tools/chain_knob_probe.py > gpurun_out/chain_knobs_${T}.log 2>&1 || { tail -20 gpurun_out/chain_knobs_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/chain_knobs_${T}.log
