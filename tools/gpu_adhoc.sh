#!/bin/bash
# scratch GPU session (edited per experiment; the checkpoints use tools/gpu_checkpoint.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04n
CHAIN_SETS=shard0/8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_shard_$T -o run -- python3 tools/chain_knob_probe.py > gpurun_out/tl_shard_$T.log 2>&1 || { tail gpurun_out/tl_shard_$T.log; exit 1; }
python3 tools/kernel_timeline.py gpurun_out/tl_shard_$T chain_rows > gpurun_out/chain_shard_timeline_$T.txt
tail -45 gpurun_out/chain_shard_timeline_$T.txt
