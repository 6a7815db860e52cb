#!/bin/bash
# scratch GPU session (edited per experiment; the checkpoints use tools/gpu_checkpoint.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_checkpoint.sh r04b tests || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/chainshard_r04b -o run -- python3 tools/chain_shard_probe.py > gpurun_out/chainshard_r04b.log 2>&1 || { tail -20 gpurun_out/chainshard_r04b.log; exit 1; }
grep -v amdgpu gpurun_out/chainshard_r04b.log
CHAIN_OF=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/chainfull_r04b -o run -- python3 tools/chain_shard_probe.py > gpurun_out/chainfull_r04b.log 2>&1 || { tail -20 gpurun_out/chainfull_r04b.log; exit 1; }
grep -v amdgpu gpurun_out/chainfull_r04b.log
bash tools/gpu_lds.sh r04b
