#!/bin/bash
# round-5 GPU call zw: chain split resolution fused into one launch per pass (resolve_tiles):
# the chain GPU tests, the fused / separate A/B on the four chain sets, the small 1/8 shard timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05zw}
timeout -k 10 400 python -u -m pytest tests/test_chain.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/chain_tests_${T}.log 2>&1 || { tail -30 gpurun_out/chain_tests_${T}.log; exit 1; }
tail -3 gpurun_out/chain_tests_${T}.log
CHAIN_SETS=s_shard0/8,small,shard0/8,large CHAIN_CONFIGS=";GB_CHAIN_FUSED=0" \
  timeout -k 10 400 python -u tools/chain_knob_probe.py > gpurun_out/chain_fused_${T}.log 2>&1 || { tail -20 gpurun_out/chain_fused_${T}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/chain_fused_${T}.log
TAG=${T} bash tools/gpu_r05zv.sh
