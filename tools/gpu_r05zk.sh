#!/bin/bash
# round-5 GPU call zk: chain split knobs re-swept on the current code ('large' and its 1/8 shard)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zk}
CHAIN_SETS=shard0/8,large CHAIN_CONFIGS="${CFG:-;GB_CHAIN_SPLIT=-1,16;GB_CHAIN_SPLIT=-1,48;GB_CHAIN_SPLIT=-1,32,0,448;GB_CHAIN_SPLIT=-1,32,0,640;GB_CHAIN_SPLIT=1024;GB_CHAIN_SPLIT=4096;GB_CHAIN_SPLIT=768}" \
  timeout -k 10 600 python -u tools/chain_knob_probe.py > gpurun_out/chain_knobs_${T}.log 2>&1 || { tail -20 gpurun_out/chain_knobs_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/chain_knobs_${T}.log
